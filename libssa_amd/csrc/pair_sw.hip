// pair_sw.hip -- the SW instantiations of pair_kernel (pair_kernel.h): main
// strips of 2*np rows, a tail strip of 2*npt rows (npt a multiple of 4 up to
// np, or 0).
#include "pair_kernel.h"

namespace ssa {

hipError_t launch_pair_sw(const StripArgs& a, int np, int npt, size_t lds_bytes, hipStream_t st, int* occ) {
    switch (np) {
    case 24: return launch_pair_np<24, false>(a, npt, lds_bytes, st, occ);
    case 32: return launch_pair_np<32, false>(a, npt, lds_bytes, st, occ);
    case 36: return launch_pair_np<36, false>(a, npt, lds_bytes, st, occ);
    case 40: return launch_pair_np<40, false>(a, npt, lds_bytes, st, occ);
    case 16: return launch_pair_np<16, false>(a, npt, lds_bytes, st, occ);
    case 8: return launch_pair_np<8, false>(a, npt, lds_bytes, st, occ);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace ssa
