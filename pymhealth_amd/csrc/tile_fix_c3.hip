// Fixed-window register-tile kernels for C = 3 (tile_idx.hip.h, FIX = true): rolling_apply
// windows of up to kIdxWmax samples at any step (launch_tile_fix, tile_idx_c3.hip).
#include "tile_idx.hip.h"

namespace mhf {
template int launch_tile_idx_c<3, true>(const IdxTileArgs& a, hipStream_t stream);
}  // namespace mhf
