"""CPU check of the algebra behind long16_kernel's row scan (kernels.hip
long16_rows): one SW row scored 64 columns at a time from the
row above -- H(r-1, j) and the F into row r, as a long16 pass leaves them in
its scratch row -- through a prefix maximum of a~(j) = a(j) + (j+1)|R| instead
of the sequential E recurrence.  Restated in numpy against the plain
recurrence (E and F clamped at 0, as long16 clamps them); the kernel itself is
checked against the oracle by tests/test_gpu_parity.py::test_long16_row_scan."""
import numpy as np


def _sw_rows(q, d, M, Q, R):
    m, n = len(q), len(d)
    H = np.zeros((m + 1, n + 1), np.int64)
    E = np.zeros((m + 1, n + 1), np.int64)
    F = np.zeros((m + 2, n + 1), np.int64)
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            E[i, j] = max(E[i, j - 1] + R, H[i, j - 1] + Q + R, 0)
            F[i, j] = max(F[i - 1, j] + R, H[i - 1, j] + Q + R, 0)
            H[i, j] = max(H[i - 1, j - 1] + M[q[i - 1], d[j - 1]], E[i, j], F[i, j], 0)
    for j in range(1, n + 1):                 # F into the row below the last
        F[m + 1, j] = max(F[m, j] + R, H[m, j] + Q + R, 0)
    return H, F


def _row_scan(hup, fin, qr, d, M, Q, R, chunk):
    """One row from H of the row above and F into this row, chunk columns per
    step (the kernel: 64 lanes), carrying lane 0's diagonal input and the
    running maximum across steps.  Returns H and the F into the next row."""
    n, rabs = len(d), -R
    h_out = np.zeros(n, np.int64)
    f_out = np.zeros(n, np.int64)
    carry_m = carry_h = 0
    for c0 in range(0, n, chunk):
        js = np.arange(c0, min(n, c0 + chunk))
        hu, f = hup[js], fin[js]
        hd = np.concatenate([[carry_h], hu[:-1]])
        carry_h = hu[-1]
        av = np.maximum(np.maximum(hd + M[qr, d[js]], f), 0)
        off = (js + 1) * rabs
        at = av + off
        pm = np.maximum.accumulate(at)
        ex = np.concatenate([[carry_m], np.maximum(carry_m, pm[:-1])])
        carry_m = max(carry_m, pm[-1])
        h = np.maximum(at, Q + ex) - off
        h_out[js] = h
        f_out[js] = np.maximum(np.maximum(f + R, h + Q + R), 0)
    return h_out, f_out


def test_row_scan_equals_the_recurrence():
    rng = np.random.default_rng(2)
    for _ in range(150):
        m, n = int(rng.integers(2, 7)), int(rng.integers(1, 150))
        Q, R = -int(rng.integers(0, 12)), -int(rng.integers(0, 5))
        M = rng.integers(-6, 12, (4, 4))
        q, d = rng.integers(0, 4, m), rng.integers(0, 4, n)
        H, F = _sw_rows(q, d, M, Q, R)
        r0 = int(rng.integers(1, m))          # rows r0 .. m-1 (0-based) by the scan
        hup, fin = H[r0, 1:].copy(), F[r0 + 1, 1:].copy()
        best = int(H[: r0 + 1].max())
        for r in range(r0, m):
            hup, fin = _row_scan(hup, fin, q[r], d, M, Q, R, int(rng.choice([1, 3, 64])))
            assert (hup == H[r + 1, 1:]).all() and (fin == F[r + 2, 1:]).all(), (Q, R, r)
            best = max(best, int(hup.max()))
        assert best == int(H.max())
