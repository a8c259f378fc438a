// support.cpp -- configuration, messages, alphabets, translation and the
// reference's top-k heap semantics.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace ssa {

Config& cfg() {
    static Config c;
    return c;
}

// ---------------------------------------------------------------- messages
bool trace_on() {
    static const bool on = getenv("SSA_AMD_TRACE") != nullptr;
    return on;
}

void fatal(const char* fmt, ...) {
    if (fmt) {
        va_list ap;
        va_start(ap, fmt);
        vfprintf(stderr, fmt, ap);
        va_end(ap);
        fputc('\n', stderr);
    }
    fflush(stdout);
    exit(1);
}

static void emit(int level, const char* prefix, bool newline, const char* fmt, va_list ap) {
    if (level > cfg().output_mode) return;
    fputs(prefix, stdout);
    vfprintf(stdout, fmt, ap);
    if (newline) fputc('\n', stdout);
}

void print_info(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    emit(OUTPUT_INFO, "libssa INFO: ", false, fmt, ap);
    va_end(ap);
}
void print_warning(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    emit(OUTPUT_WARNING, "libssa WARNING: ", true, fmt, ap);
    va_end(ap);
}
void print_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    emit(OUTPUT_ERROR, "libssa ERROR: ", true, fmt, ap);
    va_end(ap);
}

// --------------------------------------------------------------- alphabets
// Residue code order of the reference alphabets (util_sequence.c:40-88):
// amino acids "-ABCDEFGHIKLMNPQRSTVWXYZU*OJ" (0..27, '-' itself unmapped),
// nucleotides "-ACMGRSVTWYHKDBN" (0..15, IUPAC bit masks, U == T, '-' -> 0).
static const char kAA[] = "-ABCDEFGHIKLMNPQRSTVWXYZU*OJ";
static const char kNT[] = "-ACMGRSVTWYHKDBN";

namespace {
struct Maps {
    signed char aa[256], nt[256];
    Maps() {
        std::memset(aa, -1, sizeof aa);
        std::memset(nt, -1, sizeof nt);
        for (int c = 1; kAA[c]; c++) {
            aa[(unsigned char)kAA[c]] = (signed char)c;
            if (kAA[c] >= 'A' && kAA[c] <= 'Z') aa[(unsigned char)(kAA[c] + 32)] = (signed char)c;
        }
        for (int c = 0; kNT[c]; c++) {
            nt[(unsigned char)kNT[c]] = (signed char)c;
            if (kNT[c] >= 'A' && kNT[c] <= 'Z') nt[(unsigned char)(kNT[c] + 32)] = (signed char)c;
        }
        nt['U'] = nt['u'] = nt['T'];
    }
};
const Maps& maps() {
    static Maps m;
    return m;
}
}  // namespace

const signed char* map_aa() { return maps().aa; }
const signed char* map_nt() { return maps().nt; }

// complement of an IUPAC bit mask: swap A<->T (1<->8) and C<->G (2<->4)
uint8_t nt_complement(uint8_t c) {
    c &= 15;
    return (uint8_t)(((c & 1) << 3) | ((c & 8) >> 3) | ((c & 2) << 1) | ((c & 4) >> 1));
}

void revcompl(const uint8_t* in, size_t len, uint8_t* out) {
    for (size_t i = 0; i < len; i++) out[i] = nt_complement(in[len - 1 - i]);
}

// ------------------------------------------------------------- translation
// NCBI genetic codes 1..25 (util_sequence.c code[]), codon index over TCAG.
static const char* kCodes[25] = {
    "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNKKSS**VVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCWWTTTTPPPPHHQQRRRRIIMMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNKKSSSSVVVVAAAADDEEGGGG",
    "FFLLSSSSYYQQCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    nullptr,
    nullptr,
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNNKSSSSVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCCWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CC*WLLLSPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNKKSSGGVVVVAAAADDEEGGGG",
    "FFLLSSSSYYY*CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNNKSSSSVVVVAAAADDEEGGGG",
    "FFLLSSSSYY*QCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY*LCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    nullptr,
    nullptr,
    nullptr,
    nullptr,
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIMMTTTTNNNKSSSSVVVVAAAADDEEGGGG",
    "FFLLSS*SYY*LCC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FF*LSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCWWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSSKVVVVAAAADDEEGGGG",
    "FFLLSSSSYY**CCGWLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG"};

bool gencode_valid(int code) { return code >= 1 && code <= 23 && kCodes[code - 1]; }

static uint8_t g_qtrans[4096], g_dtrans[4096];

// An IUPAC codon (three bit masks) translates to the amino acid all its
// concrete codons agree on; D/N mixes give B, E/Q mixes give Z, anything
// else X (util_sequence.c:200-262).
static void build_table(int code, uint8_t* table) {
    const char* ct = kCodes[code - 1];
    static const int base_of_bit[4] = {2, 1, 3, 0};   // bit 0=A,1=C,2=G,3=T -> TCAG index
    for (int a = 0; a < 16; a++)
        for (int b = 0; b < 16; b++)
            for (int c = 0; c < 16; c++) {
                char aa = '-';
                for (int i = 0; i < 4; i++) {
                    if (!(a & (1 << i))) continue;
                    for (int j = 0; j < 4; j++) {
                        if (!(b & (1 << j))) continue;
                        for (int k = 0; k < 4; k++) {
                            if (!(c & (1 << k))) continue;
                            char x = ct[base_of_bit[i] * 16 + base_of_bit[j] * 4 + base_of_bit[k]];
                            if (aa == '-' || aa == x) aa = x;
                            else if (aa == 'B' && (x == 'D' || x == 'N')) {}
                            else if ((aa == 'D' || aa == 'N') && (x == 'B' || x == 'D' || x == 'N')) aa = 'B';
                            else if (aa == 'Z' && (x == 'Q' || x == 'E')) {}
                            else if ((aa == 'E' || aa == 'Q') && (x == 'Z' || x == 'Q' || x == 'E')) aa = 'Z';
                            else aa = 'X';
                        }
                    }
                }
                if (aa == '-') aa = 'X';
                table[256 * a + 16 * b + c] = (uint8_t)map_aa()[(unsigned char)aa];
            }
}

void init_translation(int q_gencode, int d_gencode) {
    build_table(q_gencode, g_qtrans);
    build_table(d_gencode, g_dtrans);
}

// us_translate_sequence (util_sequence.c:334-382): codons read forward from
// `frame`, or on the reverse complement starting `frame` from the end.
std::vector<uint8_t> translate(bool db_side, const uint8_t* dna, size_t len, int strand, int frame) {
    const uint8_t* t = db_side ? g_dtrans : g_qtrans;
    size_t plen = len > (size_t)frame ? (len - frame) / 3 : 0;
    std::vector<uint8_t> out(plen + 1, 0);
    if (strand == 0) {
        size_t pos = frame;
        for (size_t p = 0; p < plen; p++, pos += 3)
            out[p] = t[((dna[pos] & 15) << 8) | ((dna[pos + 1] & 15) << 4) | (dna[pos + 2] & 15)];
    } else {
        size_t pos = len - 1 - frame;
        for (size_t p = 0; p < plen; p++, pos -= 3)
            out[p] = t[(nt_complement(dna[pos]) << 8) | (nt_complement(dna[pos - 1]) << 4) |
                       nt_complement(dna[pos - 2])];
    }
    return out;
}

// -------------------------------------------------------------------- top-k
// minheap_add (minheap.c:75-91): sift-up with strict '<'; when full the root
// is replaced only by a strictly larger score, then sifted down preferring
// the right child only when it is strictly smaller (minheap.c:50-73).
bool TopK::add(const Hit& h) {
    if (k_ == 0) return false;
    if (a_.size() < k_) {
        size_t i = a_.size();
        a_.push_back(h);
        while (i > 0) {
            size_t p = (i - 1) / 2;
            if (!(h.score < a_[p].score)) break;
            a_[i] = a_[p];
            i = p;
        }
        a_[i] = h;
        return true;
    }
    if (!(a_[0].score < h.score)) return false;
    size_t p = 0, c = 1, n = a_.size();
    while (c < n) {
        if (c + 1 < n && a_[c + 1].score < a_[c].score) c++;
        if (!(a_[c].score < h.score)) break;
        a_[p] = a_[c];
        p = c;
        c = 2 * p + 1;
    }
    a_[p] = h;
    return true;
}

void sort_hits(std::vector<Hit>& v) {
    std::sort(v.begin(), v.end(), [](const Hit& x, const Hit& y) {
        if (x.score != y.score) return x.score > y.score;
        return x.id > y.id;
    });
}

std::vector<Hit> TopK::sorted() const {
    std::vector<Hit> v(a_);
    sort_hits(v);
    return v;
}

}  // namespace ssa
