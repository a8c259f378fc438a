/*
 * libssa_extern_db.h -- the database plugin contract consumed by libssa.
 *
 * Same ABI as the reference src/libssa_extern_db.h:28-56, which the
 * reference links against the (unvendored) libsdb.  This repository ships
 * its own provider, libssa_fasta_db.so (libssa_amd/csrc/fasta_db.cpp):
 *   - record index = ID (0-based, in file order),
 *   - multi-line records joined, whitespace dropped, residues kept as ASCII,
 *   - empty records kept with seqlen 0 (so IDs stay aligned; the search
 *     skips them, reference db_adapter.c:231-233),
 *   - ssa_db_get_sequence(id) returns NULL when id >= count.
 * libssa_amd.so only calls these four symbols, so a third-party libsdb can
 * be linked in its place.
 */
#ifndef LIBSSA_EXTERN_DB_H_
#define LIBSSA_EXTERN_DB_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    size_t ID;
    size_t seqlen;
    char * seq;
} seqinfo_t;

typedef seqinfo_t * p_seqinfo;

int ssa_db_init( const char * db_name );          /* reference libssa_extern_db.h:39 */
size_t ssa_db_get_sequence_count( void );         /* :44 */
p_seqinfo ssa_db_get_sequence( size_t id );       /* :49 */
void ssa_db_close( void );                        /* :56 */

#ifdef __cplusplus
}
#endif

#endif /* LIBSSA_EXTERN_DB_H_ */
