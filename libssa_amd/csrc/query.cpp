// query.cpp -- query construction (reference src/query.c:42-264) and the
// per-search query buffers (src/algo/searcher.c:42-90).
#include <cstdio>
#include <cstring>
#include <string>

#include "common.h"

namespace ssa {

// Maps with the alphabet fixed at creation; unknown symbols are dropped and
// reported unless they are '\n', ' ' or '\t' (query.c:102-130).
static SeqBuf map_query(const char* s, size_t len, const signed char* map) {
    SeqBuf out;
    out.seq.reserve(len + 1);
    std::string unknown;
    for (size_t i = 0; i < len; i++) {
        signed char m = map[(unsigned char)s[i]];
        if (m >= 0) out.seq.push_back((uint8_t)m);
        else if (s[i] != '\n' && s[i] != ' ' && s[i] != '\t') unknown.push_back(s[i]);
    }
    if (!unknown.empty())
        print_warning("%ld unknown symbols found and removed: '%s'", (long)unknown.size(), unknown.c_str());
    out.seq.push_back(0);
    return out;
}

static void fill(p_query q, const char* s, size_t len) {
    int st = cfg().symtype;
    const signed char* map = (st == AMINOACID || st == TRANS_DB) ? map_aa() : map_nt();
    SeqBuf orig = map_query(s, len, map);
    if (st == NUCLEOTIDE) {
        q->nt[0] = orig;
        if (cfg().strands & 2) {
            // MI355X: the reverse complement has the mapped length (the
            // reference sizes it by the raw text length, query.c:139-143)
            q->nt[1].seq.assign(orig.seq.size(), 0);
            revcompl(orig.seq.data(), orig.len(), q->nt[1].seq.data());
        }
    } else if (st == TRANS_QUERY || st == TRANS_BOTH) {
        for (int strand = 0; strand < 2; strand++) {
            if (!((strand + 1) & cfg().strands)) continue;
            for (int f = 0; f < 3; f++) q->aa[3 * strand + f].seq = translate(false, orig.seq.data(), orig.len(), strand, f);
        }
    } else {
        q->aa[0] = orig;
    }
}

static p_query make() {
    p_query q = new _query();
    q->symtype = cfg().symtype;
    return q;
}

p_query query_from_string(const char* s) {
    p_query q = make();
    fill(q, s, strlen(s));
    return q;
}

// First FASTA record only; the header line (if any) is kept without '>'.
p_query query_from_file(const char* path) {
    if (strcmp(path, "-") == 0) {
        print_error("Query not specified");
        return nullptr;
    }
    FILE* f = fopen(path, "r");
    if (!f) {
        print_error("Cannot open query file: %s", path);
        return nullptr;
    }
    std::string line, seq, header;
    auto getl = [&](std::string& out) -> bool {
        out.clear();
        int c;
        bool any = false;
        while ((c = fgetc(f)) != EOF) {
            any = true;
            out.push_back((char)c);
            if (c == '\n') break;
        }
        return any;
    };
    if (!getl(line)) {
        print_error("Could not initialise from query sequence");
        fclose(f);
        return nullptr;
    }
    p_query q = make();
    if (!line.empty() && line[0] == '>') {
        header = line.substr(1);
        if (!header.empty() && header.back() == '\n') header.pop_back();
        q->header = header;
        if (!getl(line)) {
            print_error("Could not read first line from query sequence");
            delete q;
            fclose(f);
            return nullptr;
        }
    }
    for (;;) {
        if (line.empty() || line[0] == '>') break;
        seq += line;
        if (!getl(line)) break;
    }
    fclose(f);
    fill(q, seq.data(), seq.size());
    return q;
}

std::vector<QueryView> query_views(p_query q) {
    std::vector<QueryView> v;
    int st = cfg().symtype;
    auto add = [&](SeqBuf& b, int strand, int frame) {
        if (b.seq.empty()) b.seq.push_back(0);
        v.push_back({b.seq.data(), b.len(), strand, frame, (char*)b.seq.data()});
    };
    if (st == NUCLEOTIDE) {
        for (int s = 0; s < 2; s++)
            if ((s + 1) & cfg().strands) add(q->nt[s], s, 0);
    } else if (st == AMINOACID || st == TRANS_DB) {
        add(q->aa[0], 0, 0);
    } else {
        for (int s = 0; s < 2; s++)
            if ((s + 1) & cfg().strands)
                for (int f = 0; f < 3; f++) add(q->aa[3 * s + f], s, f);
    }
    return v;
}

}  // namespace ssa
