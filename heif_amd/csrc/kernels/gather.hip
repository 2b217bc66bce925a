// gather.hip — k_gather_tiles: the single-image tile split across GPUs
// (SURVEY §8(e), config 5 "1->8 GPUs") ends with every rank's tiles copied into
// one device's full-size planes.  Grid tiles are independent pictures
// (src/heic/decoder.rs:98-119 decodes them one by one), so the gather is a
// plain 2-D window copy per selected tile; the source planes may be another
// device's memory (a peer pointer, or one mapped from another process with
// heifgpu_ipc_open), read over xGMI by this kernel.
//
// Mapping: one launch for all selected tiles and planes: blockIdx.z = plane,
// blockIdx.y = selected tile, blockIdx.x = group of 4 rows, 64 threads per row
// each moving 16 bytes per step (a 512-sample 16-bit row is 1 KiB = one step
// of the 64 threads).  HBM/xGMI-bound: every byte is read once and written
// once.
#include "kernels.hpp"

namespace hg {

#if !defined(HG_HOST_EMU)
namespace {

__global__ void __launch_bounds__(256) k_gather_tiles(GatherArgs g) {
    const int c = (int)blockIdx.z;
    const int k = g.offset + (int)blockIdx.y * g.stride;
    if (c >= g.planes || k >= g.n_tiles) return;
    const int sx = c ? g.sx : 0, sy = c ? g.sy : 0;  // chroma subsampling (log2)
    const int pw = (g.W + (1 << sx) - 1) >> sx, ph = (g.H + (1 << sy) - 1) >> sy;
    const int x0 = ((k % g.cols) * g.tw) >> sx, y0 = ((k / g.cols) * g.th) >> sy;
    if (x0 >= pw || y0 >= ph) return;  // a tile wholly inside the crop
    const int w = min(g.tw >> sx, pw - x0), h = min(g.th >> sy, ph - y0);
    const int y = (int)blockIdx.x * 4 + (int)threadIdx.y;
    if (y >= h) return;
    const size_t wb = (size_t)w * (size_t)g.bps;
    const uint8_t *s = reinterpret_cast<const uint8_t *>(g.src[c]) + (size_t)(y0 + y) * (size_t)g.spitch[c] +
                       (size_t)x0 * (size_t)g.bps;
    uint8_t *d = reinterpret_cast<uint8_t *>(g.dst[c]) + (size_t)(y0 + y) * (size_t)g.dpitch[c] +
                 (size_t)x0 * (size_t)g.bps;
    const bool al = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15u) == 0;
    for (size_t o = (size_t)threadIdx.x * 16; o < wb; o += 64 * 16) {
        if (al && o + 16 <= wb) {
            *reinterpret_cast<uint4 *>(d + o) = *reinterpret_cast<const uint4 *>(s + o);
        } else {
            const size_t e = o + 16 < wb ? o + 16 : wb;
            for (size_t b = o; b < e; ++b) d[b] = s[b];
        }
    }
}

}  // namespace

hipError_t launch_gather_tiles(const GatherArgs &g, hipStream_t s) {
    if (g.n_tiles <= 0 || g.stride <= 0 || g.offset >= g.stride) return hipErrorInvalidValue;
    const int sel = (g.n_tiles - g.offset + g.stride - 1) / g.stride;
    if (sel <= 0) return hipSuccess;
    const dim3 grid((unsigned)((g.th + 3) / 4), (unsigned)sel, (unsigned)g.planes);
    hipLaunchKernelGGL(k_gather_tiles, grid, dim3(64, 4), 0, s, g);
    return hipGetLastError();
}
#endif

}  // namespace hg
