/*
 * libssa_amd.h -- MI355X-specific extensions to the libssa C ABI.
 *
 * Everything in libssa.h works unchanged; these entry points add what a
 * sharded, multi-GPU deployment needs and what the benchmark measures:
 *
 *   - ssa_amd_search(..., SSA_AMD_LOG) scores the locally opened DB (a shard
 *     whose IDs start at ssa_amd_set_id_offset()) and returns its top-k
 *     INSERTION LOG: the exact subset of (score, id) pairs that the
 *     reference's min-heap (src/util/minheap.c:75-91) would ever accept when
 *     fed this shard in ID order.  Any element the global heap accepts is in
 *     its shard's log, so concatenating the logs in shard order and calling
 *     ssa_amd_replay() reproduces the 64-bit single-thread reference result
 *     bit for bit, including the IDs chosen among equal scores.  Logs are a
 *     few hundred elements, so one gather over RCCL/xGMI is all the
 *     cross-GPU traffic a search needs.
 *   - ssa_amd_get_stats() exposes HIP-event kernel times and counters.
 */
#ifndef LIBSSA_AMD_H_
#define LIBSSA_AMD_H_

#include <stdint.h>
#include <stddef.h>
#include "libssa.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int64_t score;
    uint64_t db_id;      /* global DB ID (local ID + id offset) */
    uint8_t query_id;    /* index into the query's strand/frame buffers */
    uint8_t db_strand;
    uint8_t db_frame;
    uint8_t pad[5];
} ssa_hit_t;             /* 24 bytes, like the reference's elem_t */

typedef struct {
    double search_ms;    /* host wall time of the last search call */
    double kernel_ms;    /* HIP-event time of the int16 strip kernels */
    double wide_ms;      /* HIP-event time of the exact int64 re-score kernel */
    double d2h_ms;       /* device->host score copy (HIP events) */
    double replay_ms;    /* host top-k replay */
    double pack_ms;      /* DB packing + upload (only when the DB changed) */
    uint64_t cells;      /* sum over queries of qlen * sum of entry lengths */
    uint64_t entries;    /* DB entries scored per query */
    uint64_t overflow_8; /* reference-style counters (manager.c:157-160) */
    uint64_t overflow_16;
    uint64_t wide_count; /* entries re-scored exactly by the int64 kernel */
    uint32_t kernel_launches;
    int32_t device;
    uint64_t kernel_bytes;   /* algorithmic HBM bytes of the strip kernels */
    char kernel[32];         /* main scoring kernel of the last search, e.g. "pair_f16_sw" */
} ssa_amd_stats_t;

#define SSA_AMD_SW 0
#define SSA_AMD_NW 1
#define SSA_AMD_TOPK 0      /* sorted top-k, as sw_align/nw_align */
#define SSA_AMD_LOG 1       /* insertion log in replay order */

int ssa_amd_device_count( void );
void ssa_amd_set_device( int device );
void ssa_amd_set_id_offset( size_t offset );
int ssa_amd_prepare_db( void );            /* pack + upload the DB now; returns 0 on success */
void ssa_amd_get_stats( ssa_amd_stats_t * out );
void ssa_amd_set_option( const char * name, long value );

/* Scores the open DB against the query.  mode: SSA_AMD_TOPK or SSA_AMD_LOG.
 * Returns the number of hits written (at most cap; the log never exceeds
 * the number of DB entries). */
size_t ssa_amd_search( p_query query, int algo, size_t hitcount, int bit_width, int mode,
                       ssa_hit_t * out, size_t cap );

/* Replays an insertion log (concatenated shard logs, in shard order) and
 * writes the sorted top-k (score desc, id desc).  Returns the count. */
size_t ssa_amd_replay( const ssa_hit_t * log, size_t n, size_t hitcount, ssa_hit_t * out );

#ifdef __cplusplus
}
#endif

#endif /* LIBSSA_AMD_H_ */
