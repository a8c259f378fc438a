// matrices.cpp -- scoring matrix state with the reference's semantics
// (src/matrices.c:335-568): a 32 x 32 int64 table indexed [db code][query
// code], every cell the matrix text does not set is -1, row/column symbols of
// a text matrix are mapped with the AMINO-ACID map even for nucleotide work,
// constant scoring fills codes >= 1 only.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>

#include "common.h"

namespace ssa {

#include "builtin_matrices.inc"

Matrix& matrix() {
    static Matrix m;
    return m;
}

static void reset() {
    Matrix& M = matrix();
    for (int i = 0; i < kDim * kDim; i++) M.m[i] = -1;
    M.ready = true;
}

void matrix_free() { matrix().ready = false; }

void matrix_constant(int match, int mismatch) {
    reset();
    Matrix& M = matrix();
    M.constant = true;
    for (int a = 1; a < kDim; a++)
        for (int b = 1; b < kDim; b++) M.m[(a << 5) + b] = (a == b) ? match : mismatch;
}

// One line of the NCBI text format (matrices.c:388-437): '#'/blank lines are
// comments, a line starting with blank/tab lists the column symbols, every
// other line is "<row symbol> <score> <score> ...".
struct TextParser {
    int nsym = 0;
    std::vector<int> order;
    void line(const char* s) {
        const signed char* map = map_aa();
        char c = s[0];
        if (c == '\n' || c == '#' || c == 0) return;
        if (c == ' ' || c == '\t') {
            size_t k = 0;
            for (const char* p = s + 1; *p; p++) {
                if (*p == ' ' || *p == '\t' || *p == '\n') continue;
                if (k < order.size()) order[k] = map[(unsigned char)*p];
                else order.push_back(map[(unsigned char)*p]);
                k++;
                nsym++;
            }
            return;
        }
        int a = map[(unsigned char)c];
        const char* p = s + 1;
        for (int i = 0; i < nsym; i++) {
            char* end = nullptr;
            long v = strtol(p, &end, 10);
            if (end == p) {
                // sscanf matching failure is fatal in the reference; an early
                // end of line leaves the remaining cells untouched
                const char* q = p;
                while (*q == ' ' || *q == '\t' || *q == '\n' || *q == '\r') q++;
                if (*q) fatal("Problem parsing score matrix file.");
                break;
            }
            int b = i < (int)order.size() ? order[i] : -1;
            if (a >= 0 && b >= 0 && a < kDim && b < kDim) matrix().m[(a << 5) + b] = v;
            p = end;
        }
    }
};

void matrix_from_string(const char* text) {
    if (!text) fatal("Cannot read score matrix string.");
    reset();
    TextParser tp;
    const char* s = text;
    std::string line;
    while (*s) {
        const char* nl = strchr(s, '\n');
        size_t n = nl ? (size_t)(nl - s) : strlen(s);
        line.assign(s, n);
        tp.line(line.c_str());
        s = nl ? nl + 1 : s + n;
    }
}

void matrix_from_file(const char* path) {
    FILE* f = fopen(path, "r");
    if (!f) fatal("Cannot open score matrix file.");
    reset();
    TextParser tp;
    char buf[2048];
    while (fgets(buf, sizeof buf, f)) tp.line(buf);
    fclose(f);
}

void matrix_builtin(const char* name) {
    for (int k = 0; k < 8; k++) {
        if (strcasecmp(name, kBuiltinNames[k]) == 0) {
            reset();
            Matrix& M = matrix();
            for (int x = 0; x < 28; x++)
                for (int y = 0; y < 28; y++) M.m[(x << 5) + y] = kBuiltin[k][28 * x + y];
            return;
        }
    }
    fatal("Unknown matrix: %s", name);
}

}  // namespace ssa
