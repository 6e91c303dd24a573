// mr_internal.h — entry points shared between the engine's translation units
// (not part of the C ABI in include/mr_engine.h).
#ifndef MR_INTERNAL_H
#define MR_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "mr_engine.h"

namespace mr_internal {

// k_topk_merge of n_shards [shard][n_te][k] device lists into [n_te][k] outputs,
// enqueued on the context's stream (no host wait).
int merge_async(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const int32_t* songs_in,
                const int64_t* keys_in, int32_t* songs_out, int64_t* keys_out, double* scores_out);

// The same over G gathered record blocks (keys [n_te*k] int64 at byte 0,
// songs [n_te*k] int32 at byte 8*n_te*k, block stride rec_bytes).
int merge_records_async(mr_ctx* c, int32_t n_shards, int32_t n_te, int32_t k, const void* records, int64_t rec_bytes,
                        int32_t* songs_out, int64_t* keys_out, double* scores_out);

// The context's own top-k record block (the exchange's send buffer; valid
// until mr_load / mr_destroy) and its size in bytes.
int topk_records(mr_ctx* c, void** records, int64_t* rec_bytes);

// mr_load's input checks (CSR shapes, sorted rows, id ranges, counts) without
// loading: what mr_group_load runs before it reads the dataset itself.
int validate_dataset(const mr_dataset* d);

// Synchronous device -> host copy of rows (pitched), staged through the
// context's pinned buffers when the destination is large pageable memory.
int d2h_staged(mr_ctx* c, void* dst, size_t dpitch, const void* src, size_t spitch, size_t row_bytes, size_t rows);

// Number of contexts of one process that share this context's device (set
// by mr_group_load before mr_load, default 1): the lazily allocated neighbour
// lists' budget (free device memory / 8 at load) is divided by it, since the
// group's contexts measure free memory at once, before any of them allocates.
int set_device_share(mr_ctx* c, int n);

// Set the calling thread's mr_last_error() message; returns code.
int set_error(int code, const char* msg);

}  // namespace mr_internal

#endif  // MR_INTERNAL_H
