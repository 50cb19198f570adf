// Indexed register-tile kernels for C = 3 (see tile_idx.hip.h), and the host side of
// the indexed tile path. One TU per channel count so the unrolled kernels build in parallel.
#include "tile_idx.hip.h"

namespace mhf {

template int launch_tile_idx_c<3, false>(const IdxTileArgs& a, hipStream_t stream);
extern template int launch_tile_idx_c<1, false>(const IdxTileArgs& a, hipStream_t stream);
extern template int launch_tile_idx_c<1, true>(const IdxTileArgs& a, hipStream_t stream);
extern template int launch_tile_idx_c<3, true>(const IdxTileArgs& a, hipStream_t stream);
static_assert(kTileFixWmax == kIdxWmax, "tile_idx.h");

bool tile_idx_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, fmask_t mask,
                 const float* x) {
    if (mask & ~kTileIdxBits) return false;
    if (!(channels == 1 || channels == 3)) return false;
    if (sample_stride != channels) return false;
    if (channels > 1 && ch_stride != 1) return false;
    return reinterpret_cast<uintptr_t>(x) % 4 == 0;
}

int launch_tile_idx(const IdxTileArgs& a, hipStream_t stream) {
    if (!a.x || !a.out || !a.starts || !a.ends || a.nwin < 1 || a.feats.n < 1)
        return MHF_EINVAL;
    if (a.channels == 3) return launch_tile_idx_c<3, false>(a, stream);
    if (a.channels == 1) return launch_tile_idx_c<1, false>(a, stream);
    return MHF_EINVAL;
}

// fixed windows: the x pointer's 4-B alignment is checked at launch
bool tile_fix_ok(int32_t channels, int64_t ch_stride, int64_t sample_stride, int64_t wsize,
                 fmask_t mask) {
    if (wsize < 1 || wsize > kIdxWmax) return false;
    const float* aligned = reinterpret_cast<const float*>(uintptr_t(256));
    return tile_idx_ok(channels, ch_stride, sample_stride, mask, aligned);
}

int launch_tile_fix(const IdxTileArgs& a, hipStream_t stream) {
    if (!a.x || !a.out || a.nwin < 1 || a.feats.n < 1 || a.wsize < 1 || a.wsize > kIdxWmax ||
        a.wstep < 1 || a.first < 0 || reinterpret_cast<uintptr_t>(a.x) % 4 != 0)
        return MHF_EINVAL;
    // every window inside the record (the caller's nw formula, windows.py:86)
    if ((a.first + a.nwin - 1) * a.wstep + a.wsize > a.n_samples) return MHF_EINVAL;
    if (a.channels == 3) return launch_tile_idx_c<3, true>(a, stream);
    if (a.channels == 1) return launch_tile_idx_c<1, true>(a, stream);
    return MHF_EINVAL;
}

}  // namespace mhf
