// Host check of the fp32 tower wave-stream schedule (csrc/hip/tower32_sched.h):
// every (column block, k-group) fragment has a distinct position inside the
// layer's stream, pair units and leftover segments sit where the kernel's
// traversal (tower32.hip t32_layer) reads them, and each wave's leftover range
// spans at most kT32MaxSeg blocks.  Prints "ok" or the first failure.
#include <cstdio>
#include <set>
#include <vector>

#include "hip/tower32_sched.h"

using namespace pbx;

int main() {
  for (int ncol = 1; ncol <= 40; ++ncol)
    for (int ng = 1; ng <= 40; ++ng) {
      const T32Sched s = t32_sched(ncol, ng);
      const int64_t total = t32_stream_groups(ncol, ng);
      std::set<int64_t> seen;
      for (int c = 0; c < ncol; ++c)
        for (int g = 0; g < ng; ++g) {
          const int64_t p = t32_group_pos(ncol, ng, c, g);
          if (p < 0 || p >= total || !seen.insert(p).second) {
            printf("FAIL ncol %d ng %d: (%d, %d) -> %lld (total %lld)\n", ncol, ng, c, g, (long long)p,
                   (long long)total);
            return 1;
          }
        }
      // the kernel's traversal: wave w reads its units, then its segments
      for (int w = 0; w < kT32Waves; ++w) {
        int64_t st = t32_wave_off(s, ng, w);
        for (int u = 0; u < s.q; ++u) {
          const int col = 2 * (u * kT32Waves + w);
          for (int g = 0; g < ng; ++g)
            for (int j = 0; j < 2; ++j)
              if (t32_group_pos(ncol, ng, col + j, g) != 2 * (st + g) + j) {
                printf("FAIL unit ncol %d ng %d w %d u %d\n", ncol, ng, w, u);
                return 1;
              }
          st += t32_ceil_ring(ng);
        }
        const int lo = t32_rem_lo(s, w), hi = t32_rem_lo(s, w + 1);
        int seg = 0;
        for (int f = lo; f < hi; ++seg) {
          const int j = f / ng, g0 = f - j * ng;
          const int len = (ng - g0) < (hi - f) ? (ng - g0) : (hi - f);
          for (int i = 0; i < len; ++i)
            if (t32_group_pos(ncol, ng, 8 * s.q + j, g0 + i) != 2 * (st + i / 2) + (i & 1)) {
              printf("FAIL seg ncol %d ng %d w %d\n", ncol, ng, w);
              return 1;
            }
          st += t32_seg_steps(len);
          f += len;
        }
        if (seg > kT32MaxSeg) {
          printf("FAIL ncol %d ng %d: wave %d has %d segments\n", ncol, ng, w, seg);
          return 1;
        }
        if (st != t32_wave_off(s, ng, w + 1)) {
          printf("FAIL ncol %d ng %d: wave %d stream length\n", ncol, ng, w);
          return 1;
        }
      }
    }
  printf("ok\n");
  return 0;
}
