// Streaming save of the host + SSD tiers (tier_save.cc).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../common/ckpt_format.h"
#include "tier_store.h"

namespace pbx {

struct TierSaveStats {
  int64_t rows = 0, host_rows = 0, ssd_rows = 0;
  double total_s = 0;
};

// kind 0: batch model (keys_path / vals_path .npy), kind 1: xbox text
// (keys_path); rows of embedding width `dim` (make_row_layout(dim) fields)
// and the tiers' stride.  Either tier may be null.  saved_mixed (optional)
// receives the mixed keys of every saved row.
TierSaveStats save_tiers(HostTier* host, SsdLog* ssd, int kind, const SaveSelect& sel, int dim,
                         float embedx_threshold, const std::string& keys_path, const std::string& vals_path,
                         int threads, std::vector<uint64_t>* saved_mixed);

}  // namespace pbx
