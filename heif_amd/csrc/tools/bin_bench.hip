// bin_bench.hip — micro-benchmark of k_parse's CABAC engine (tuning only).
// Includes parse.hip so it measures exactly the product's dec_bin /
// dec_bypass / next_byte / ensure_bytes, on a synthetic byte stream.
//   build: make -C heif_amd/csrc bin_bench ; run: heif_amd/csrc/build/bin_bench [waves_per_simd]
#include "../kernels/parse.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace hg {
namespace {
__global__ void __launch_bounds__(256) k_binbench(const uint8_t *bits, uint32_t len, int nbins, int mode,
                                                  uint32_t *out, uint64_t *cycles) {
    __shared__ WaveLds lds[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    Parser p;
    p.w = &lds[wave];
    p.lane = lane;
    p.status = 0;
    p.src = bits + (size_t)blockIdx.x * 64;
    p.nal_end = len - (uint32_t)blockIdx.x * 64 - 64;
    p.flags = 0;
    p.cx.load_tables(lane);
    p.cx.init(lane, 30);
    engine_init(p, 0);
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < nbins; i += 16) {
        ensure_bytes(p);
        if (mode == 0) {
#pragma unroll
            for (int k = 0; k < 16; ++k) acc += dec_bin(p, CTX_SIG + (k & 7));
        } else if (mode == 1) {
#pragma unroll
            for (int k = 0; k < 16; ++k) acc += dec_bypass(p);
        } else {
            // data-dependent context choice, like sig_coeff_flag
            int c = 0;
            for (int k = 0; k < 16; ++k) {
                int b = dec_bin(p, CTX_SIG + c);
                acc += b;
                c = (c + 1 + b) & 15;
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[blockIdx.x * 4 + wave] = acc + p.status;
        atomicAdd((unsigned long long *)cycles, (unsigned long long)(t1 - t0));
    }
}
}  // namespace
}  // namespace hg

int main(int argc, char **argv) {
    const int wps = argc > 1 ? atoi(argv[1]) : 1;  // waves per SIMD
    const int nbins = 200000;
    const uint32_t len = 64u << 20;
    std::vector<uint8_t> h(len);
    uint64_t x = 88172645463325252ull;
    for (auto &b : h) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        b = (uint8_t)x;
    }
    uint8_t *d;
    uint32_t *out;
    uint64_t *cyc;
    hipMalloc(&d, len);
    hipMemcpy(d, h.data(), len, hipMemcpyHostToDevice);
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 8);
    const int blocks = 256 * wps;  // 1 block = 4 waves = 1 wave per SIMD of one CU
    for (int mode = 0; mode < 3; ++mode) {
        hipMemset(cyc, 0, 8);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(hg::k_binbench, dim3(blocks), dim3(256), 0, 0, d, len, nbins, mode, out, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        uint64_t c;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        const double waves = blocks * 4.0;
        printf("mode %d (%s): waves/SIMD %d  %.1f memtime-cycles/bin/wave  %.2f Gbins/s chip\n", mode,
               mode == 0 ? "ctx bins" : mode == 1 ? "bypass" : "ctx, dependent ctxInc", wps,
               (double)c / waves / nbins, waves * nbins / (ms * 1e-3) / 1e9);
    }
    return 0;
}
