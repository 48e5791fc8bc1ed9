// Instance-parser plugin ABI: user parsers shipped as shared objects and
// loaded with dlopen, chosen per dataset by `set_so_parser_name`.
//
// Behaviour reproduced (not code): the reference's ISlotParser plugin contract
// (fw/data_feed.h:1964-2015 -- Init(slots), ParseOneInstance(line, GetInsFunc)
// which may emit any number of instances per line; loader SlotInsParserMgr
// data_feed.cc:3604-3670).  The reference ABI passes C++ objects
// (SlotRecord, std::function) across the .so boundary; ours is a plain C ABI
// so a plugin needs no headers beyond this one and no matching C++ runtime.
//
// A plugin exports three symbols:
//
//   void* pbx_parser_create(int nslots, const char* const* slot_names,
//                           const char* slot_types);   // 'u' uint64 / 'f' float
//   int   pbx_parser_parse_line(void* parser, const char* line, size_t len,
//                               const pbx_ins_sink* sink);
//         -> number of instances emitted (0 = line dropped), < 0 = parse error
//   void  pbx_parser_destroy(void* parser);
//
// (sink fields appended after `commit` are NULL-checked by a plugin that uses
// them; plugins built against the 4-callback struct keep working.)
//
// For every instance the plugin calls `add_u64` / `add_f32` for the slots it
// has values for (slot = index into the slot list given at create time; the
// values of slots the dataset does not use are discarded by the host),
// optionally `set_meta`, then `commit`.  `parse_line` is called concurrently
// from the loader threads with the same parser handle, so it must be
// re-entrant (keep per-line state on the stack).
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pbx_ins_sink {
  void* ctx;
  void (*add_u64)(void* ctx, int slot, const uint64_t* v, int n);
  void (*add_f32)(void* ctx, int slot, const float* v, int n);
  void (*set_meta)(void* ctx, const char* ins_id, int ins_id_len, uint64_t search_id, uint32_t cmatch,
                   uint32_t rank);
  // returns 1 if the instance was kept (it has at least one sparse feasign)
  int (*commit)(void* ctx);
  // GPU replica cache feed (reference SlotPaddleBoxDataFeedWithGpuReplicaCache):
  // append one cache row, get its offset to store as the instance's feasign.
  // NULL when the dataset has no replica cache attached.
  int64_t (*add_cache)(void* ctx, const float* v, int n);
  // input-index feed (reference InputIndexDataFeed): offset of a string key in
  // the input table (UINT64_MAX when absent).  NULL when no table is attached.
  uint64_t (*index_offset)(void* ctx, const char* key, int len);
} pbx_ins_sink;

// Optional 4th symbol for index files (reference ParseIndexData):
//   int pbx_parser_parse_index(void* parser, const char* line, size_t len,
//                              const pbx_index_sink* sink);  -> entries added
typedef struct pbx_index_sink {
  void* ctx;
  void (*add_index)(void* ctx, const char* key, int key_len, const float* v, int n);
} pbx_index_sink;

// Optional 5th symbol, UnrollInstance (reference ISlotParser::UnrollInstance
// data_feed.h:1994-1998, run on the loaded pass when
// FLAGS_padbox_dataset_enable_unrollinstance, data_set.cc:2275-2277,2825):
//   int64_t pbx_parser_unroll(void* parser, const pbx_record_view* view,
//                             const pbx_ins_sink* sink);
// The plugin reads the pass's records through `view` (slot = index into the
// slot list given at create time; unused slots read as empty) and emits the
// pass's NEW record set through `sink` -- any number of instances per input
// record.  Returns the number emitted (< 0 = error: the pass is kept as is).
typedef struct pbx_record_view {
  void* ctx;
  int64_t n;  // records in the pass
  int (*get_u64)(void* ctx, int64_t rec, int slot, const uint64_t** v);  // -> count
  int (*get_f32)(void* ctx, int64_t rec, int slot, const float** v);     // -> count
  void (*get_meta)(void* ctx, int64_t rec, const char** ins_id, int* ins_id_len, uint64_t* search_id,
                   uint32_t* cmatch, uint32_t* rank);
} pbx_record_view;

// Optional 6th symbol, whole-file parsing (reference
// ISlotParser::ParseFileInstance, data_feed.cc:3850-3870), used for every file
// when FLAGS_enable_ins_parser_file is set:
//   int64_t pbx_parser_parse_file(void* parser, const char* path,
//                                 pbx_read_fn read, void* read_ctx,
//                                 const pbx_ins_sink* sink);
// The plugin pulls the (decompressed / converted) file bytes with
// read(read_ctx, buf, len) -> bytes read, 0 at end of file, and emits
// instances through `sink`.  `path` is the file name when
// FLAGS_enable_ins_parser_add_file_path is set, else NULL.  Returns the
// number of instances emitted, < 0 on a parse error.
typedef int64_t (*pbx_read_fn)(void* read_ctx, char* buf, int64_t len);

typedef void* (*pbx_parser_create_fn)(int, const char* const*, const char*);
typedef int (*pbx_parser_parse_line_fn)(void*, const char*, size_t, const pbx_ins_sink*);
typedef void (*pbx_parser_destroy_fn)(void*);
typedef int (*pbx_parser_parse_index_fn)(void*, const char*, size_t, const pbx_index_sink*);
typedef int64_t (*pbx_parser_unroll_fn)(void*, const pbx_record_view*, const pbx_ins_sink*);
typedef int64_t (*pbx_parser_parse_file_fn)(void*, const char*, pbx_read_fn, void*, const pbx_ins_sink*);

#ifdef __cplusplus
}
#endif
