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
    double wide_ms;      /* HIP-event time of the exact re-score tier (0 under option "lean_events") */
    double d2h_ms;       /* device filter + result copy (HIP events; 0 under "lean_events") */
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
    double prep_ms;          /* host work before the first kernel launch (profiles, uploads) */
    double upload_ms;        /* device time of the per-search uploads before the first kernel (0 under
                                option "lean_events") */
    double sync_wait_ms;     /* host time blocked in the final stream synchronisation */
    uint32_t strip_rows;     /* pair kernel: rows of its main strips (2 x "pair_np"); 0: other kernels */
    uint32_t counters;       /* 1: overflow_8/16 were computed (bit width 64, output mode >= OUTPUT_INFO
                                or option "counters" 1); 0: not computed, they read 0 */
    uint32_t long_entries;   /* lanes (64 per group) of the longest groups scored by a long-entry kernel (view 0) */
    char long_kernel[24];    /* that kernel: "long16_rl<R>" (packed 16-bit SW), "long32_w<W>_rl<R>" (int32;
                                "+"-joined when split over two launches), "" none */
    uint32_t part_retries;   /* searches run again without strip parts because a part's wait for its
                                group's first part ran into option "part_wait_us" (results unaffected) */
    /* running totals since the library was loaded (never reset): a caller
     * times N searches by two reads, with no call between the searches */
    uint64_t total_searches;
    double total_kernel_ms;  /* sum of kernel_ms */
    double total_search_ms;  /* sum of search_ms */
    uint64_t filter_candidates;  /* scores of the last search the device top-k filter let through to
                                    the host (every score when it ran without the filter) */
    double gather_ms;        /* host wall time of this rank's last ssa_amd_gather_logs (staging, the
                                collective, rank 0's replay) */
    uint32_t gather_rounds;  /* 1: the slot gather alone; 2: this rank also sent (or rank 0 received)
                                log rows beyond the 512-row slot point to point */
    uint32_t rare_merged;    /* DB residue codes the last search scored through one upper-bound class
                                (option "rare_merge"; 0: none) */
    uint32_t rare_rescored;  /* entries holding one of them that the device filter forwarded and the
                                int32 tier re-scored exactly */
    uint32_t slots;          /* device slots of the last search (1: one device; more: SSA_AMD_DEVICES or
                                ssa_amd_set_devices, one host thread per slot) */
    int32_t slot_device[16];     /* per slot: its HIP device */
    double slot_kernel_ms[16];   /* per slot: HIP-event time of its DP kernels */
    double slot_search_ms[16];   /* per slot: host time of its device search and shard replay */
    uint32_t graph;          /* slot 0's last search: 0 issued call by call, 1 captured into a new HIP graph,
                                2 replayed the cached graph (option "graph") */
} ssa_amd_stats_t;

#define SSA_AMD_SW 0
#define SSA_AMD_NW 1
#define SSA_AMD_TOPK 0      /* sorted top-k, as sw_align/nw_align */
#define SSA_AMD_LOG 1       /* insertion log in replay order */

/* Devices.  An unchanged libssa caller searches on every visible GPU, as
 * the reference uses every core by default (src/util/thread_pool.c:42,
 * get_nprocs()): at the first init_db, unless ssa_amd_set_device(s) was
 * called before, the library reads the environment variable
 *   SSA_AMD_DEVICES = all (also: unset or empty) | current | 0,2,...
 * -- every visible device, the current HIP device only, or this list
 * (repeats allowed: several slots on one device).  Several devices work as
 * ssa_amd_set_devices below.  set_thread_count(n) (libssa.h: the reference's
 * number of search workers) caps that list at its first n devices (0: all),
 * so the reference's thread sweeps become device sweeps.  An explicit
 * ssa_amd_set_device(s) always wins (one rank per GPU:
 * ssa_amd_set_device(local_rank)) and no thread count changes it. */
int ssa_amd_device_count( void );
void ssa_amd_set_device( int device );
void ssa_amd_set_id_offset( size_t offset );
/* Search on several devices from this one process (one persistent host
 * thread per device slot inside sw_align / nw_align -- the caller's thread
 * drives slot 0 -- the DB split into contiguous record ranges at chunk_size
 * boundaries, balanced by residues, the slots' insertion logs merged in
 * slot order; results identical to a single device).  n = 0 returns to
 * single-device mode (ssa_amd_set_device).  Returns 0, or 1 for an invalid
 * device list. */
int ssa_amd_set_devices( const int * devices, int n );
/* The device slots the next search uses (after SSA_AMD_DEVICES, which is
 * read here if init_db has not read it yet): writes up to cap device ids to
 * out (may be NULL) and returns the slot count. */
int ssa_amd_get_devices( int * out, int cap );
int ssa_amd_prepare_db( void );            /* pack + upload the DB now; returns 0 on success */
void ssa_amd_get_stats( ssa_amd_stats_t * out );
/* Tuning knobs (results never change, only which kernel computes them):
 *   "strip_np" 8|16|32   int16 strip kernels: packed rows per strip
 *   "pair_np" 0|16|24|32|36|40  pair kernel main strip of 2 x pair_np rows; 0 (default):
 *                        SW 24, NW the tallest of 40/32/24 whose pair table lets
 *                        two workgroups share a CU (36 is SW only)
 *   "sw_kernel" 0|1      1: int16 strip kernel instead of the pair kernel
 *   "force_wide" 0|1     1: every entry through the int64 kernel
 *   "no_filter" 0|1      1: copy every score back (no device top-k filter)
 *   "long_groups" -1|0|N leading groups scored one entry per wave: auto, never, N
 *   "long_share_pct" P   auto threshold: P % of one SIMD's share of all columns
 *   "long_waves" 0|4|1   waves scoring one long entry (its query rows split over
 *                        them): auto (4 for groups beyond "long4_share_pct", 1
 *                        for the rest), always 4, always 1
 *   "long4_share_pct" P  auto: 4 waves per entry for groups longer than P % of
 *                        one SIMD's share of all columns (default 1500: where one
 *                        wave's latency would outlast the pair kernel)
 *   "long16" 1|0         SW long entries on packed 16-bit patterns, one wave
 *                        per entry, whenever min(m, n) x max score fits (default);
 *                        0: the int32 kernel ("long_waves" applies to it)
 *   "filter_prefix_regs" 1|0  the top-k filter's block scan with its states in registers and
 *                        merges at the list width k needs, for DBs of <= 256 filter blocks
 *                        (default), or always the general scan
 *   "graph" 0|1          1: a single-view search with the device filter and no overflow counters runs
 *                        as cached HIP graphs -- the operations between its two timing records captured
 *                        once per launch plan, replayed with the changed kernel arguments set on their
 *                        nodes (stats graph); 0 (default: the graphs measured slower than the direct
 *                        calls): every stream operation issued on its own
 *   "upload_kernel" 1|0  1 (default): the per-search upload block (matrix, boundary, query) is read
 *                        from pinned host memory by a kernel on the search's stream; 0: a
 *                        copy-engine transfer (hipMemcpyAsync)
 *   "tier_defer" 1|0     single-view searches: the exact re-score tier runs only when the device
 *                        filter's header reports overflowed lanes, after the result's copy
 *                        (default 1); 0: always, between the DP kernels and the filter
 *   "tail_rows4" 1|0     the pair kernel's last strip at 4-row granularity (default; SW 48-row and
 *                        NW 64/80-row strips, after a main strip), or 8-row (0)
 *   "long_prio" 1|0      long16 waves at raised issue priority over the pair waves (default 1)
 *   "long_pad" 1|0       long-entry workgroups pad their LDS to the pair kernel's, so a finished one
 *                        leaves a pair workgroup's hole (default 1; 0 measured -6 % on the Swiss-Prot form)
 *   "filter_onepass" 1|0 the device top-k filter as one launch (a decoupled look-back over its
 *                        blocks; default 1) or as three (block maxima, prefix, select)
 *   "long_latency" 1|0   a DB of at most 256 groups (16 384 entries), a query of two strips or more:
 *                        every group goes to the long-entry kernels when their throughput estimate
 *                        beats the pair wave's latency (default 1; one 513-residue entry, q = 390:
 *                        SW 1.48 -> 0.14 ms); 0: the length rules alone
 *   "plan_cache" 1|0     a search with the query and settings of one of the last four reuses
 *                        their plan (residue classes, bounds, strips; default 1); 0: plan each search
 *   "long_gate" 1|0|P    the pair kernel starts after the long-entry workgroups have (default 1;
 *                        0: no wait, the long-entry streams' priority alone orders them; 2..99:
 *                        after the first P % of them)
 *   "long16_rows" 1|0|2  queries beyond 1 024 rows: long16 passes planned by issue cost, up to 8
 *                        last rows scored by a row scan (default 1); 0: RL 16 passes; 2: the
 *                        cost model at every query length (q = 513: RL 8 + 1 scanned row)
 *   "pair_prio_groups" 0|-1|N  pair-kernel groups (longest first) at raised
 *                        wave priority: none (default), one per SIMD, N
 *   "timeline" 0|1       1: record every DP wave's start/end (ssa_amd_get_timeline)
 *   "pair_ticket" 1|0    pair-kernel workgroups take the next groups in start order
 *                        (an atomic ticket; default) or in blockIdx order
 *   "pair_parts" 0|1|2|3 pair-kernel groups run as 2 (or 3) dependent work units of
 *                        consecutive strips (all groups' first parts, then all second
 *                        parts, ...), so the launch ends on small units: 0 (default) 2
 *                        for groups of at least 4 strips, 1 never, 2 always, 3 three
 *   "rescore32" 1|0      entries the DP kernels cannot score exactly (overflow) are re-scored
 *                        by the int32 long-entry kernel, one wave per entry, whenever int32 is
 *                        exact for the DB (default); 0: always the int64 kernel
 *   "part_wait_us" N     bound of a strip part's wait for its group's first part (default
 *                        2000000); a timed-out wait makes the search run again without parts
 *                        (stats part_retries), results unchanged
 *   "rare_merge" 0|1     1 (default 0): when a query's residue classes leave the pair table too big
 *                        for three workgroups per CU, the rarest classes share one class scoring
 *                        the maximum of their rows, and the entries holding them that the device
 *                        filter forwards are re-scored exactly (stats rare_merged / rare_rescored)
 *   "filter_host" 0..3   the device filter's result through a D2H copy (0, default) or written by
 *                        the filter into pinned host memory (1: system-scope release, 2: system-
 *                        scope stores, the host spinning on a sequence word; 3: plain stores,
 *                        published by the end of the dispatch, the host synchronising as usual)
 *   "sync_spin" 1|0      1 (default): the host thread spins while a search runs (hipDeviceScheduleSpin,
 *                        set at the library's first pack on a device; 15 us less between two
 *                        searches); 0: HIP's own scheduling (yields the core).  The flag is
 *                        PROCESS-WIDE for that device: every HIP user of the process (e.g. torch)
 *                        then spins in its own synchronisations too, and a search keeps one host
 *                        core busy for its whole duration.  It only takes effect when the library
 *                        is the first to use the device in the process (a context made before keeps
 *                        its flags); set 0 before the first init_db to leave the flags alone
 *   "lean_events" 1|0    1 (default): no timing markers around the upload, the re-score tier
 *                        and the filter (stats upload_ms, wide_ms, d2h_ms read 0; kernel_ms
 *                        kept; C2 +0.5 %, profiles/r05/ab/lean_events); 0: all markers
 *   "side_tier" 0|1      1: the int32 re-score tier runs beside the device filter on a second
 *                        stream instead of in front of it (default 0: no gain measured)
 *   "pair_split" P       strip parts for every quad of groups (0, default) or only the first P %
 *                        (the longest, P > 0) or the last -P % (P < 0)
 *   "counters" -1|0|1    the reference's 8/16-bit overflow counters (stats overflow_8/16,
 *                        m_run's INFO line): -1 (default) only at output mode
 *                        OUTPUT_INFO, where the reference prints them; 0 never; 1 always
 * Unknown names print a warning. */
void ssa_amd_set_option( const char * name, long value );

/* The last search's wave timeline (option "timeline"; of the last query view
 * for multi-view searches): rows of 4 uint32 --
 *   pair_kernel: (group, start, end, place); long_kernel: (0x80000000 | lane
 *   of its entry, start, end, place)
 * start/end in s_memrealtime ticks (100 MHz, low 32 bits), place = XCC << 16 |
 * HW_ID[15:0].  Rows never written stay zero.  Copies at most cap rows to out
 * (may be NULL) and returns the row count.  A profiling aid (tools/timeline.py),
 * not part of the reference's interface. */
size_t ssa_amd_get_timeline( uint32_t * out, size_t cap );

/* Scores the open DB against the query.  mode: SSA_AMD_TOPK or SSA_AMD_LOG.
 * Returns the number of hits written (at most cap; the log never exceeds
 * the number of DB entries). */
size_t ssa_amd_search( p_query query, int algo, size_t hitcount, int bit_width, int mode,
                       ssa_hit_t * out, size_t cap );

/* Several queries against the open DB in one call.
 * Query i's sorted top-k goes to out[i * hitcount ...], its length to
 * counts[i]; returns the total.  Each query is exactly sw_align/nw_align's
 * result.  The DB is packed once and stays in HBM; per query the library
 * adds ~0.1 ms of fixed work (profile upload, filter, replay) to the DP,
 * which is VALU-bound, so there is no DB streaming for a batch to amortise
 * (DESIGN.md §7). */
size_t ssa_amd_search_batch( const p_query * queries, size_t nq, int algo, size_t hitcount, int bit_width,
                             ssa_hit_t * out, size_t * counts );

/* Replays an insertion log (concatenated shard logs, in shard order) and
 * writes the sorted top-k (score desc, id desc).  Returns the count. */
size_t ssa_amd_replay( const ssa_hit_t * log, size_t n, size_t hitcount, ssa_hit_t * out );

/* Multi-process search over RCCL (one process per GPU).  The
 * reference merges its worker threads' heaps in one process
 * (src/algo/manager.c:141-145); a sharded deployment merges the shards'
 * insertion logs instead:
 *   rank 0:        ssa_amd_dist_unique_id(id)   (id: ssa_amd_dist_unique_id_bytes()
 *                  bytes, handed to the other ranks out of band -- MPI, a TCP
 *                  store, a shared file)
 *   every rank:    ssa_amd_set_device(local GPU); ssa_amd_dist_init(rank, world, id)
 *   every search:  n = ssa_amd_search(q, algo, k, width, SSA_AMD_LOG, log, cap);
 *                  c = ssa_amd_gather_logs(log, n, k, out)   (collective)
 * ssa_amd_gather_logs gathers every rank's log over RCCL (one ncclGather of
 * fixed 512-row slots to rank 0; a log longer than its slot sends the rest of
 * its rows to rank 0 point to point, ncclSend / ncclRecv between those two
 * ranks only) and on rank 0 writes the global sorted top-k to out and returns
 * its length -- bit-identical to one process searching the whole DB; other
 * ranks return 0.  ssa_amd_dist_init returns 0 on success.
 * ssa_amd_merge_logs is rank 0's merge alone: nlogs logs at rows + r * stride
 * (counts[r] rows each), replayed in order through the reference heap. */
int ssa_amd_dist_unique_id( void * id );
size_t ssa_amd_dist_unique_id_bytes( void );
/* Local readiness, no communication: 0 when RCCL resolves and this rank's
 * device can be selected, i.e. everything ssa_amd_dist_init checks before it
 * enters the collective ncclCommInitRank.  Agree on it across ranks (e.g. a
 * MIN all-reduce) before calling ssa_amd_dist_init, so that no rank waits in
 * the init for a peer that gave up. */
int ssa_amd_dist_available( void );
int ssa_amd_dist_init( int rank, int world, const void * id );
/* Test support: the calling THREAD becomes rank `rank` of an in-process
 * group of `world` threads (keyed by `group`), whose collectives exchange
 * through host memory instead of RCCL -- the same slot layout, count rows and
 * point-to-point remainder as over RCCL.  Released by ssa_amd_dist_finalize on
 * that thread.  Returns 0 on success. */
int ssa_amd_dist_init_fake( int rank, int world, int group );
/* Ranks of the current communicator (ncclCommCount), 0 before init. */
int ssa_amd_dist_ranks( void );
void ssa_amd_dist_finalize( void );
size_t ssa_amd_gather_logs( const ssa_hit_t * log, size_t n, size_t hitcount, ssa_hit_t * out );
size_t ssa_amd_merge_logs( const ssa_hit_t * rows, const size_t * counts, size_t nlogs, size_t stride,
                           size_t hitcount, ssa_hit_t * out );
/* Residue-balanced contiguous shards: cuts records
 * [0, n) with the given lengths into `world` ID ranges
 * [bounds[r], bounds[r + 1]) (bounds has world + 1 entries, bounds[0] = 0,
 * bounds[world] = n) whose residue sums are as equal as cuts at multiples of
 * `align` allow (align = chunk_size keeps a multi-view search's chunk-
 * interleaved insertion order the concatenation of the shards' orders;
 * 0 or 1 = any record).  The multi-process analogue of ssa_amd_set_devices'
 * split.  Returns 0, or 1 for world < 1. */
int ssa_amd_shard_bounds( const uint64_t * lengths, size_t n, size_t world, size_t align, size_t * bounds );

/* Persistent packed DB: ssa_amd_save_db writes the device
 * layout of the open DB (packing it first if needed); ssa_amd_load_db,
 * called after init_db on the same DB file and with the same
 * init_symbol_translation settings, uploads that layout instead of
 * re-reading, mapping and packing every record.  The file records symbol
 * type, strands, DB genetic code and record count and is refused when they
 * differ.  Both return 0 on success. */
int ssa_amd_save_db( const char * path );
int ssa_amd_load_db( const char * path );

/* COMPUTE_ALIGNMENT traceback of one (query, DB sequence) pair of mapped
 * codes with the current matrix and gap penalties (reference align.c +
 * cigar.c, the same routine sw_align/nw_align use for their hits).  Writes
 * region = {query begin, query end, db begin, db end} and the NUL-terminated
 * CIGAR (truncated to cap - 1 characters); returns the CIGAR length. */
size_t ssa_amd_align_pair( int algo, const char * query, size_t qlen, const char * db, size_t dlen,
                           size_t region[4], char * cigar, size_t cap );

/* The query buffers a search scores for the current symbol type and strands
 * (reference searcher.c:42-90): one q_seq_t per strand/frame view, codes as
 * handed out in alignment_t.query.seq.  Writes up to cap views; returns the
 * number of views. */
size_t ssa_amd_query_views( p_query query, q_seq_t * out, size_t cap );

/* Translates mapped nucleotide codes (map_ncbi_nt16 values) with the query
 * (db_side = 0) or DB (db_side = 1) genetic code chosen by
 * init_symbol_translation, strand 0 (forward) or 1 (reverse complement),
 * frame 0..2 -- reference util_sequence.c:332-382.  Writes min(result, cap)
 * amino-acid codes; returns the protein length (len - frame) / 3, 0 when
 * len < frame. */
size_t ssa_amd_translate( int db_side, const char * nt_codes, size_t len, int strand, int frame,
                          char * out, size_t cap );

#ifdef __cplusplus
}
#endif

#endif /* LIBSSA_AMD_H_ */
