// fasta_db.cpp -- libssa_fasta_db.so, the DB plugin shipped with libssa_amd
// (contract: include/libssa_extern_db.h, reference src/libssa_extern_db.h).
//
// The reference links an unvendored libsdb; its behaviour at this boundary is
// pinned by the reference's tests (tests/test_libssa_extern_db.c:12-55):
// record index == ID, NULL past the end, sequence count of the file.  Records
// keep their residues as ASCII with line breaks and other whitespace removed;
// empty records stay (seqlen 0) so later IDs do not shift.
//
// The file is memory-mapped and parsed in parallel: it is cut into one
// piece per thread at record starts ("\n>"), each piece is parsed into its
// own residue arena, and the arenas are concatenated in order -- the result
// is byte-identical to a sequential pass.  A 10 M-record shard takes well
// under a second per init_db.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "bulk_alloc.h"
#include "libssa_extern_db.h"

namespace {
struct FastaDB {
    ssa::Chars arena;                   // (no zeroing resize, huge pages: bulk_alloc.h)
    std::vector<seqinfo_t> recs;
};
FastaDB* g_db = nullptr;

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// Parses [p, end): records start at '>' at a line start; residues of the
// lines that follow a header, whitespace dropped.  Text before the first
// header is ignored.  `first_in_record` is set when the piece starts inside
// a record (never: pieces are cut at record starts, except piece 0).
struct Piece {
    ssa::Chars res;
    std::vector<size_t> offs;   // record starts in res
};

void parse_piece(const char* p, const char* end, bool at_line_start, Piece& out) {
    bool in_rec = false;
    while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* le = nl ? nl : end;
        if (at_line_start && *p == '>') {
            out.offs.push_back(out.res.size());
            in_rec = true;
        } else if (in_rec) {
            // (uninitialised growth: the line's bytes are written right here)
            const size_t base = out.res.size();
            out.res.resize(base + (size_t)(le - p));
            char* w = out.res.data() + base;
            for (const char* q = p; q < le; q++)
                if (!is_space(*q)) *w++ = *q;
            out.res.resize((size_t)(w - out.res.data()));
        }
        at_line_start = true;
        p = nl ? nl + 1 : end;
    }
}

bool load(const char* path, FastaDB& db) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat stt;
    if (fstat(fd, &stt) != 0) { close(fd); return false; }
    const size_t sz = (size_t)stt.st_size;
    const char* buf = nullptr;
    if (sz > 0) {
        void* m = mmap(nullptr, sz, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { close(fd); return false; }
        madvise(m, sz, MADV_SEQUENTIAL);
        buf = (const char*)m;
    }
    close(fd);
    const char* end = buf + sz;
    // cut points at record starts
    const unsigned nth = sz < (8u << 20) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<const char*> cut{buf};
    for (unsigned t = 1; t < nth; t++) {
        const char* c = std::max(cut.back(), buf + sz / nth * t);
        const char* q = c;
        while (q < end) {
            const char* nl = (const char*)memchr(q, '\n', (size_t)(end - q));
            if (!nl || nl + 1 >= end) { q = end; break; }
            if (nl[1] == '>') { q = nl + 1; break; }
            q = nl + 1;
        }
        cut.push_back(q);
    }
    cut.push_back(end);
    std::vector<Piece> pieces(nth);
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nth; t++)
        pool.emplace_back([&, t]() {
            if (cut[t] < cut[t + 1]) parse_piece(cut[t], cut[t + 1], true, pieces[t]);
        });
    for (auto& th : pool) th.join();
    if (buf) munmap((void*)buf, sz);
    // concatenate
    size_t total = 0, nrec = 0;
    std::vector<size_t> rbase(nth), obase(nth);
    for (unsigned t = 0; t < nth; t++) {
        rbase[t] = total;
        obase[t] = nrec;
        total += pieces[t].res.size();
        nrec += pieces[t].offs.size();
    }
    db.arena.resize(total + 1);
    db.recs.resize(nrec);
    pool.clear();
    for (unsigned t = 0; t < nth; t++)
        pool.emplace_back([&, t]() {
            const Piece& P = pieces[t];
            if (!P.res.empty()) memcpy(db.arena.data() + rbase[t], P.res.data(), P.res.size());
            for (size_t i = 0; i < P.offs.size(); i++) {
                const size_t b = P.offs[i];
                const size_t e = i + 1 < P.offs.size() ? P.offs[i + 1] : P.res.size();
                seqinfo_t& r = db.recs[obase[t] + i];
                r.ID = obase[t] + i;
                r.seqlen = e - b;
                r.seq = db.arena.data() + rbase[t] + b;
            }
        });
    for (auto& th : pool) th.join();
    db.arena[total] = 0;
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
