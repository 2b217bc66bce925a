// color.hip — k_ycbcr_rgb: decoded Y/Cb/Cr planes → interleaved 8-bit RGB with
// the item's irot rotation (libheif's default output).
//
// The reference stops at parsing `irot` (src/heif/grammar.rs) and never
// produces pixels; the arithmetic is H.273's (R = Y + 2(1-Kr)Cr,
// B = Y + 2(1-Kb)Cb, G = Y - (2Kb(1-Kb)Cb + 2Kr(1-Kr)Cr)/Kg, limited range
// rescaled by 255/219 and 255/224) in 16-bit fixed point with the
// coefficients rounded on the host (ColorCoefs), so a test can restate it
// exactly.  irot rotates anticlockwise by 90 degrees per unit (ISO/IEC
// 23008-12 6.5.10).  Subsampled chroma (4:2:0, 4:2:2) is replicated (nearest sample).
//
// Mapping: one thread per 4 output pixels along a row (12-byte store as
// three dwords when the row is 4-byte aligned).  HBM-bound: 1.5 bytes read
// and 3 written per pixel.
#include "kernels.hpp"

namespace hg {

#if !defined(HG_HOST_EMU)
namespace {

template <typename Pel>
__global__ void __launch_bounds__(256) k_ycbcr_rgb(ColorArgs c) {
    const int ox0 = (int)(blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int oy = (int)blockIdx.y;
    if (ox0 >= c.out_w || oy >= c.out_h) return;
    const Pel *Y = reinterpret_cast<const Pel *>(c.plane[0]);
    const Pel *Cb = reinterpret_cast<const Pel *>(c.plane[1]);
    const Pel *Cr = reinterpret_cast<const Pel *>(c.plane[2]);
    uint32_t px[4] = {0, 0, 0, 0};
    const int np = c.out_w - ox0 < 4 ? c.out_w - ox0 : 4;
    for (int k = 0; k < np; ++k) {
        const int ox = ox0 + k;
        int x, y;  // source sample (coded orientation)
        switch (c.rotation) {
        case 1: x = c.w - 1 - oy; y = ox; break;
        case 2: x = c.w - 1 - ox; y = c.h - 1 - oy; break;
        case 3: x = oy; y = c.h - 1 - ox; break;
        default: x = ox; y = oy; break;
        }
        const int ys = (int)(*reinterpret_cast<const Pel *>(reinterpret_cast<const uint8_t *>(Y) + (size_t)y * c.pitch[0]
                                                             + (size_t)x * sizeof(Pel))) >> c.shift;
        int cb = 0, cr = 0;
        if (c.chroma) {
            const int xc = x >> chroma_sx(c.chroma), yc = y >> chroma_sy(c.chroma);
            const size_t o1 = (size_t)yc * c.pitch[1] + (size_t)xc * sizeof(Pel);
            const size_t o2 = (size_t)yc * c.pitch[2] + (size_t)xc * sizeof(Pel);
            cb = ((int)*reinterpret_cast<const Pel *>(reinterpret_cast<const uint8_t *>(Cb) + o1) >> c.shift) - 128;
            cr = ((int)*reinterpret_cast<const Pel *>(reinterpret_cast<const uint8_t *>(Cr) + o2) >> c.shift) - 128;
        }
        const int yv = c.ys * (ys - c.yoff);
        const int r = (yv + c.cr_r * cr + 32768) >> 16;
        const int g = (yv - c.cb_g * cb - c.cr_g * cr + 32768) >> 16;
        const int b = (yv + c.cb_b * cb + 32768) >> 16;
        const uint32_t R = (uint32_t)min(max(r, 0), 255), G = (uint32_t)min(max(g, 0), 255),
                       B = (uint32_t)min(max(b, 0), 255);
        px[k] = R | (G << 8) | (B << 16);
    }
    uint8_t *row = reinterpret_cast<uint8_t *>(c.rgb) + (size_t)oy * c.rgb_pitch + (size_t)ox0 * 3;
    if (np == 4 && !(reinterpret_cast<uintptr_t>(row) & 3)) {
        uint32_t *w = reinterpret_cast<uint32_t *>(row);
        w[0] = px[0] | (px[1] << 24);
        w[1] = (px[1] >> 8) | (px[2] << 16);
        w[2] = (px[2] >> 16) | (px[3] << 8);
    } else {
        for (int k = 0; k < np; ++k) {
            row[3 * k] = (uint8_t)px[k];
            row[3 * k + 1] = (uint8_t)(px[k] >> 8);
            row[3 * k + 2] = (uint8_t)(px[k] >> 16);
        }
    }
}

}  // namespace

hipError_t launch_ycbcr_rgb(const ColorArgs &c, int bytes_per_sample, hipStream_t s) {
    const dim3 grid((unsigned)((c.out_w + 4 * 256 - 1) / (4 * 256)), (unsigned)c.out_h);
    if (bytes_per_sample == 1) hipLaunchKernelGGL(k_ycbcr_rgb<uint8_t>, grid, dim3(256), 0, s, c);
    else hipLaunchKernelGGL(k_ycbcr_rgb<uint16_t>, grid, dim3(256), 0, s, c);
    return hipGetLastError();
}
#endif

}  // namespace hg
