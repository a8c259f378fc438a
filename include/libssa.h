/*
 * libssa.h -- public C ABI of the MI355X-native libssa engine.
 *
 * Drop-in for the reference header src/libssa.h (xubo245/libssa): every
 * constant value, struct layout and function signature below is identical,
 * so existing C callers (the reference's libssa_example.c, its benchmark
 * drivers and the public-API parts of its tests) compile and link against
 * libssa_amd.so unchanged.  Each declaration cites the reference line it
 * replaces.  Behavioural notes specific to this implementation are marked
 * "MI355X:".
 */
#ifndef LIBSSA_H_
#define LIBSSA_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (reference src/libssa.h:29-72) ---------------------------- */
#define VERBOSE_ON 1
#define VERBOSE_OFF 0

#define SIMD_ON 1
#define SIMD_OFF 0

#define BLOSUM45 "blosum45"
#define BLOSUM50 "blosum50"
#define BLOSUM62 "blosum62"
#define BLOSUM80 "blosum80"
#define BLOSUM90 "blosum90"
#define PAM30 "pam30"
#define PAM70 "pam70"
#define PAM250 "pam250"

/* symbol types */
#define NUCLEOTIDE 0
#define AMINOACID 1
#define TRANS_QUERY 2
#define TRANS_DB 3
#define TRANS_BOTH 4

/* strands */
#define FORWARD_STRAND 1
#define COMPLEMENTARY_STRAND 2
#define BOTH_STRANDS 3

/* score width: a hint on MI355X (every width returns the exact 64-bit
 * scores; the width only selects which overflow counters are reported) */
#define BIT_WIDTH_8 8
#define BIT_WIDTH_16 16
#define BIT_WIDTH_64 64

#define OUTPUT_SILENT 0
#define OUTPUT_ERROR 1
#define OUTPUT_WARNING 2
#define OUTPUT_INFO 3

#define COMPUTE_SCORE 0
#define COMPUTE_ALIGNMENT 1

#define READ_FROM_FILE 0
#define READ_FROM_STRING 1
#define MATRIX_BUILDIN 2

/* accepted for compatibility; MI355X: no effect on the GPU path */
#define COMPUTE_ON_SSE2 0
#define COMPUTE_ON_SSE41 1
#define COMPUTE_ON_AVX2 2

/* ---- data types (reference src/libssa.h:79-117) -------------------------- */
struct _query;
typedef struct _query * p_query;

typedef struct {
    char * seq;        /* internal residue codes, NUL terminated (not ASCII) */
    size_t len;
    size_t ID;         /* DB sequence ID as given by the DB plugin */
    int strand;
    int frame;
} db_seq_t;

typedef struct {
    char * seq;        /* points into the p_query: keep the query alive */
    size_t len;
    int strand;
    int frame;
} q_seq_t;

typedef struct {
    db_seq_t db_seq;
    q_seq_t query;
    char * alignment;  /* CIGAR for COMPUTE_ALIGNMENT, else NULL */
    size_t alignment_len;
    long score;
    size_t align_q_start;
    size_t align_q_end;
    size_t align_d_start;
    size_t align_d_end;
} alignment_t;
typedef alignment_t * p_alignment;

typedef struct {
    p_alignment * alignments;
    size_t len;
} alignment_list_t;
typedef alignment_list_t * p_alignment_list;

/* ---- technical initialisation (reference src/libssa.h:122-128) ----------- */
void set_output_mode( int mode );
void set_simd_compute_mode( int mode );   /* MI355X: accepted, ignored by the GPU path */
void set_chunk_size( size_t size );       /* insertion-order granularity of the top-k replay */
void set_thread_count( size_t count );    /* MI355X: host threads for DB packing */

/* ---- initialisation (reference src/libssa.h:154-227) --------------------- */
void init_score_matrix( int mode, const char * matrix );
/* NOTE: as in the reference (libssa.c:115-117) the FIRST argument is used as
 * the match score and the second as the mismatch score. */
void init_constant_scores( const int8_t p, const int8_t m );
void init_gap_penalties( const int8_t gapO, const int8_t gapE );
void init_symbol_translation( int type, int strands, int db_gencode, int q_gencode );
void init_db( const char * db_file );
p_query init_sequence_fasta( int mode, const char * fasta_seq_file );
void free_sequence( p_query p );

/* ---- alignment (reference src/libssa.h:240-263) -------------------------- */
p_alignment_list sw_align( p_query p, size_t hitcount, int bit_width, int align_type );
p_alignment_list nw_align( p_query p, size_t hitcount, int bit_width, int align_type );
void free_alignment( p_alignment_list alist );
void ssa_exit( void );

#ifdef __cplusplus
}
#endif

#endif /* LIBSSA_H_ */
