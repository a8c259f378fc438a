// fasta_db.cpp -- libssa_fasta_db.so, the DB plugin shipped with libssa_amd
// (contract: include/libssa_extern_db.h, reference src/libssa_extern_db.h).
//
// The reference links an unvendored libsdb; its behaviour at this boundary is
// pinned by the reference's tests (tests/test_libssa_extern_db.c:12-55):
// record index == ID, NULL past the end, sequence count of the file.  Records
// keep their residues as ASCII with line breaks and other whitespace removed;
// empty records stay (seqlen 0) so later IDs do not shift.
//
// The file is read with one sequential pass into a single residue arena; for
// a 10 M-record shard that is a few seconds, once per init_db.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "libssa_extern_db.h"

namespace {
struct FastaDB {
    std::vector<char> arena;
    std::vector<seqinfo_t> recs;
    std::vector<size_t> offs;
};
FastaDB* g_db = nullptr;

bool load(const char* path, FastaDB& db) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return false; }
    const long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<char> buf(sz > 0 ? (size_t)sz : 0);
    if (sz > 0 && fread(buf.data(), 1, (size_t)sz, f) != (size_t)sz) { fclose(f); return false; }
    fclose(f);
    db.arena.reserve(buf.size());
    const char* p = buf.data();
    const char* end = p + buf.size();
    bool in_rec = false;
    while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* le = nl ? nl : end;
        if (*p == '>') {
            db.offs.push_back(db.arena.size());
            in_rec = true;
        } else if (in_rec) {
            for (const char* q = p; q < le; q++) {
                const char c = *q;
                if (c != ' ' && c != '\t' && c != '\r' && c != '\v' && c != '\f') db.arena.push_back(c);
            }
        }
        p = nl ? nl + 1 : end;
    }
    db.offs.push_back(db.arena.size());
    db.arena.push_back(0);
    const size_t n = db.offs.size() - 1;
    db.recs.resize(n);
    for (size_t i = 0; i < n; i++) {
        db.recs[i].ID = i;
        db.recs[i].seqlen = db.offs[i + 1] - db.offs[i];
        db.recs[i].seq = db.arena.data() + db.offs[i];
    }
    return true;
}
}  // namespace

extern "C" {

int ssa_db_init(const char* name) {
    ssa_db_close();
    FastaDB* db = new FastaDB();
    if (!name || !load(name, *db)) {
        fprintf(stderr, "libssa_fasta_db: cannot read database file %s\n", name ? name : "(null)");
        delete db;
        return 1;
    }
    g_db = db;
    return 0;
}

size_t ssa_db_get_sequence_count(void) { return g_db ? g_db->recs.size() : 0; }

p_seqinfo ssa_db_get_sequence(size_t id) {
    if (!g_db || id >= g_db->recs.size()) return nullptr;
    return &g_db->recs[id];
}

void ssa_db_close(void) {
    delete g_db;
    g_db = nullptr;
}

}  // extern "C"
