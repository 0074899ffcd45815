// sv_xcd.h — XCD-aware workgroup -> tile order for gfx950 (8 XCDs, one L2 each).
//
// The dispatcher deals workgroups to the XCDs round-robin in dispatch order (linear block id
// mod 8), so with tile = linear id a tile's neighbours land on other XCDs' L2s.  Tiles whose
// neighbours re-read the same input (stencil halos, overlapping row bands, bilinear taps)
// instead take tile (lin mod 8) * N/8 + lin div 8 (the remainder spread over the first XCDs):
// each XCD walks a contiguous range of tiles and its co-resident waves share L2 lines.
#pragma once

#include <hip/hip_runtime.h>

namespace sv {

// (bx, by, bz) of this workgroup's tile in a grid of the launch's shape; on = false keeps the
// plain order.  Results are wave-uniform (readfirstlane: addresses derived from them stay in
// SGPRs).
__device__ __forceinline__ void xcd_tile(bool on, int& bx, int& by, int& bz) {
    const unsigned nx = gridDim.x, ny = gridDim.y;
    const unsigned n = nx * ny * gridDim.z;
    const unsigned lin = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    unsigned t = lin;
    if (on) {
        const unsigned per = n >> 3, rem = n & 7u, xcd = lin & 7u, k = lin >> 3;
        t = xcd * per + min(xcd, rem) + k;
    }
    bx = __builtin_amdgcn_readfirstlane((int)(t % nx));
    by = __builtin_amdgcn_readfirstlane((int)((t / nx) % ny));
    bz = __builtin_amdgcn_readfirstlane((int)(t / (nx * ny)));
}

}  // namespace sv
