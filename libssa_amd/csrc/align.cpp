// align.cpp -- COMPUTE_ALIGNMENT: region + CIGAR of the reported hits.
//
// Post-search work on k hits, done on the host in
// parallel over hits.  Restates the reference's traceback exactly, quirks
// included, because the CIGAR strings are part of the result callers see:
//
//  * local region (align.c:39-140): a forward int64 Gotoh pass finds the
//    first cell (DB-row-major) holding the maximum; a reverse pass from that
//    cell finds the start.  The forward pass scores M[query][db] while the
//    search and the direction pass score M[db][query] (only visible with an
//    asymmetric matrix); the reverse pass re-initialises only the first
//    b_end+1 entries of its query-indexed arrays (align.c:88-91), so the
//    rest keep the forward pass's last-row values.
//  * global region (align.c:142-151): the whole query x DB rectangle.
//  * directions (cigar.c:48-211): per cell, gap-open bits from the H
//    choice and gap-extension bits from the E/F update of the same cell.
//  * traceback (cigar.c:274-346): from the region's end while both indices
//    are inside the region; a LEFT bit (open or extend) steps along the DB
//    ('I'), else an UP bit along the query ('D'), else diagonal ('M');
//    runs become "<count><op>" with the count omitted for 1.
//
// Deviation: a local alignment whose best cell score is 0 leaves the
// reference's region uninitialised (undefined behaviour); here it is
// (0, 0, 0, 0) with an empty CIGAR.
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace ssa {

namespace {

constexpr uint8_t kGapUp = 1, kGapLeft = 2, kGapExtUp = 4, kGapExtLeft = 8;

struct Region {
    size_t a_begin = 0, a_end = 0, b_begin = 0, b_end = 0;
};

inline int64_t score(const int64_t* M, uint8_t x, uint8_t y) { return M[((size_t)x << 5) + y]; }

// a = query (columns of the reference's passes), b = DB sequence (rows)
bool local_region(const uint8_t* a, size_t an, const uint8_t* b, size_t bn, const int64_t* M, int64_t Q,
                  int64_t R, Region& rg) {
    const size_t size = std::max<size_t>(std::max(an, bn), 1);
    std::vector<int64_t> HH(size, 0), EE(size, 0);
    for (size_t j = 0; j < an; j++) {
        HH[j] = 0;
        EE[j] = Q;
    }
    int64_t best = 0;
    bool found = false;
    for (size_t i = 0; i < bn; i++) {
        int64_t h = 0, p = 0, f = Q;
        for (size_t j = 0; j < an; j++) {
            f = std::max(f, h + Q) + R;
            EE[j] = std::max(EE[j], HH[j] + Q) + R;
            h = p + score(M, a[j], b[i]);
            if (h < 0) h = 0;
            if (f > h) h = f;
            if (EE[j] > h) h = EE[j];
            p = HH[j];
            HH[j] = h;
            if (h > best) {
                best = h;
                rg.a_end = j;
                rg.b_end = i;
                found = true;
            }
        }
    }
    if (!found) return false;
    for (size_t j = 0; j <= rg.b_end; j++) {
        HH[j] = -1;
        EE[j] = -1;
    }
    int64_t cost = 0;
    for (size_t ii = rg.b_end + 1; ii-- > 0;) {
        int64_t h = -1, f = -1;
        int64_t p = ii == rg.b_end ? 0 : -1;
        for (size_t jj = rg.a_end + 1; jj-- > 0;) {
            f = std::max(f, h + Q) + R;
            EE[jj] = std::max(EE[jj], HH[jj] + Q) + R;
            h = p + score(M, a[jj], b[ii]);
            if (f > h) h = f;
            if (EE[jj] > h) h = EE[jj];
            p = HH[jj];
            HH[jj] = h;
            if (h > cost) {
                cost = h;
                rg.a_begin = jj;
                rg.b_begin = ii;
                if (cost >= best) return true;
            }
        }
    }
    fatal("Internal error in align function.");
}

std::vector<uint8_t> directions(bool nw, const uint8_t* a, size_t an, const uint8_t* b, size_t bn,
                                const int64_t* M, int64_t Q, int64_t R) {
    std::vector<uint8_t> dir(an * bn, 0);
    std::vector<int64_t> he(2 * std::max<size_t>(an, 1), 0);
    if (nw)
        for (size_t i = 0; i < an; i++) {
            he[2 * i] = Q + (int64_t)(i + 1) * R;
            he[2 * i + 1] = 2 * Q + (int64_t)(i + 2) * R;
        }
    for (size_t j = 0; j < bn; j++) {
        int64_t f = nw ? 2 * Q + (int64_t)(j + 2) * R : 0;
        int64_t h = nw ? (j == 0 ? 0 : Q + (int64_t)j * R) : 0;
        uint8_t* drow = dir.data() + an * j;
        for (size_t i = 0; i < an; i++) {
            const int64_t n = he[2 * i];
            int64_t e = he[2 * i + 1];
            uint8_t d = 0;
            h += score(M, b[j], a[i]);
            if (f > h) {
                d |= kGapUp;
                h = f;
            }
            if (e > h) {
                h = e;
                d |= kGapLeft;
            }
            if (!nw && h < 0) h = 0;
            he[2 * i] = h;
            h += Q + R;
            e += R;
            f += R;
            if (f > h) d |= kGapExtUp;
            else f = h;
            if (e > h) d |= kGapExtLeft;
            else e = h;
            he[2 * i + 1] = e;
            drow[i] = d;
            h = n;
        }
    }
    return dir;
}

std::string cigar(const std::vector<uint8_t>& dir, size_t an, const Region& rg) {
    std::vector<std::pair<char, size_t>> runs;   // traceback order (end -> begin)
    size_t i = rg.a_end, j = rg.b_end;
    while (i + 1 > 0 && j + 1 > 0 && i >= rg.a_begin && j >= rg.b_begin) {
        const uint8_t d = dir[an * j + i];
        char op;
        if (d & (kGapLeft | kGapExtLeft)) {
            j--;
            op = 'I';
        } else if (d & (kGapUp | kGapExtUp)) {
            i--;
            op = 'D';
        } else {
            i--;
            j--;
            op = 'M';
        }
        if (!runs.empty() && runs.back().first == op) runs.back().second++;
        else runs.push_back({op, 1});
    }
    std::string s;
    for (size_t r = runs.size(); r-- > 0;) {
        if (runs[r].second > 1) s += std::to_string(runs[r].second);
        s += runs[r].first;
    }
    return s;
}

}  // namespace

// Region (query begin/end, DB begin/end) and CIGAR of one (query, DB) pair.
std::string traceback(int algo, const uint8_t* q, size_t qn, const uint8_t* d, size_t dn, size_t region[4]) {
    const int64_t* M = matrix().m;
    const int64_t Q = cfg().gap_open, R = cfg().gap_extend;
    Region rg;
    if (algo == kAlgoSW) {
        if (!local_region(q, qn, d, dn, M, Q, R, rg)) {
            std::fill(region, region + 4, 0);
            return std::string();
        }
    } else {
        rg.a_begin = 0;
        rg.a_end = qn - 1;      // wraps for an empty sequence, as the reference
        rg.b_begin = 0;
        rg.b_end = dn - 1;
    }
    region[0] = rg.a_begin;
    region[1] = rg.a_end;
    region[2] = rg.b_begin;
    region[3] = rg.b_end;
    const std::vector<uint8_t> dir = directions(algo == kAlgoNW, q, qn, d, dn, M, Q, R);
    return cigar(dir, qn, rg);
}

// Fills region and CIGAR of every alignment in the list, in parallel.
void compute_alignments(p_alignment_list L, int algo) {
    const size_t n = L->len;
    if (n == 0) return;
    size_t workers = std::max<size_t>(1, std::min<size_t>(n, std::thread::hardware_concurrency()));
    if (cfg().thread_count) workers = std::min(workers, cfg().thread_count);
    auto work = [&](size_t w) {
        for (size_t i = w; i < n; i += workers) {
            p_alignment a = L->alignments[i];
            size_t rg[4];
            const std::string c = traceback(algo, (const uint8_t*)a->query.seq, a->query.len,
                                            (const uint8_t*)a->db_seq.seq, a->db_seq.len, rg);
            a->align_q_start = rg[0];
            a->align_q_end = rg[1];
            a->align_d_start = rg[2];
            a->align_d_end = rg[3];
            a->alignment = (char*)malloc(c.size() + 1);
            memcpy(a->alignment, c.c_str(), c.size() + 1);
            a->alignment_len = c.size();
        }
    };
    std::vector<std::thread> pool;
    for (size_t w = 1; w < workers; w++) pool.emplace_back(work, w);
    work(0);
    for (auto& t : pool) t.join();
}

}  // namespace ssa
