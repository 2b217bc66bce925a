// simt_bench.hip — feasibility micro-benchmark for a lane-per-substream CABAC
// engine (tuning only): every lane decodes its own synthetic byte stream,
// contexts in LDS (one 144-byte set per lane), rangeTabLps/transIdxLps in LDS.
//   build: make -C heif_amd/csrc simt_bench ; run: build/simt_bench [waves_per_cu]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../kernels/cabac.hpp"

namespace {
__constant__ uint8_t c_lps_s[256] = {HG_LPS_TABLE};
__constant__ uint8_t c_trans_s[64] = {HG_TRANS_LPS};

struct Eng {
    uint32_t range, value;
    int bits_needed;
    const uint8_t *p;
};

__device__ __forceinline__ uint32_t byte_at(Eng &e) { return *e.p++; }

__global__ void __launch_bounds__(256) k_simt(const uint8_t *bits, uint32_t stream_bytes, int nbins, int mode,
                                              uint32_t *out, unsigned long long *cycles) {
    __shared__ uint8_t ctx[256][144];
    __shared__ uint8_t lps[256];
    __shared__ uint8_t trans[64];
    const int t = threadIdx.x;
    lps[t] = c_lps_s[t];
    if (t < 64) trans[t] = c_trans_s[t];
    for (int i = 0; i < 144; ++i) ctx[t][i] = (uint8_t)((i * 7 + t) & 0x7f);
    __syncthreads();
    const size_t gid = (size_t)blockIdx.x * blockDim.x + t;
    Eng e;
    e.p = bits + gid * stream_bytes;
    e.range = 510;
    e.value = (byte_at(e) << 8) | byte_at(e);
    e.bits_needed = -8;
    uint32_t acc = 0, c = 0;
    uint8_t *my = ctx[t];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < nbins; ++i) {
        // mode 0: all lanes decode a context bin; mode 1: lanes diverge between a
        // context bin and a bypass bin by their own previous bin (like mixed syntax)
        const bool bypass = mode == 1 && (c & 1);
        int bin;
        if (!bypass) {
            const int ci = (int)(c & 63);
            const uint32_t s = my[ci];
            uint32_t st = s >> 1, mps = s & 1;
            const uint32_t l = lps[(st << 2) | ((e.range >> 6) & 3)];
            e.range -= l;
            const uint32_t scaled = e.range << 7;
            if (e.value < scaled) {
                bin = (int)mps;
                st = st < 62 ? st + 1 : st;
                if (scaled < (256u << 7)) {
                    e.range = scaled >> 6;
                    e.value <<= 1;
                    if (++e.bits_needed == 0) {
                        e.bits_needed = -8;
                        e.value |= byte_at(e);
                    }
                }
            } else {
                e.value -= scaled;
                const int nb = __builtin_clz(l) - 23;
                e.value <<= nb;
                e.range = l << nb;
                bin = (int)(mps ^ 1u);
                if (st == 0) mps ^= 1u;
                st = trans[st];
                e.bits_needed += nb;
                if (e.bits_needed >= 0) {
                    e.value |= byte_at(e) << e.bits_needed;
                    e.bits_needed -= 8;
                }
            }
            my[ci] = (uint8_t)((st << 1) | mps);
        } else {
            e.value <<= 1;
            if (++e.bits_needed >= 0) {
                e.bits_needed = -8;
                e.value |= byte_at(e);
            }
            const uint32_t scaled = e.range << 7;
            bin = e.value >= scaled;
            if (bin) e.value -= scaled;
        }
        acc += bin;
        c = c * 5 + 1 + bin;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[gid] = acc;
    if (t == 0) atomicAdd(cycles, (unsigned long long)(t1 - t0));
}
}  // namespace

int main(int argc, char **argv) {
    const int blocks_per_cu = argc > 1 ? atoi(argv[1]) : 1;
    const int blocks = 256 * blocks_per_cu, threads = 256;
    const int nbins = 20000;
    const uint32_t stream_bytes = 4096;
    const size_t len = (size_t)blocks * threads * stream_bytes;
    std::vector<uint8_t> h(len);
    uint64_t x = 88172645463325252ull;
    for (auto &b : h) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = (uint8_t)x;
    }
    uint8_t *d;
    uint32_t *out;
    unsigned long long *cyc;
    if (hipMalloc(&d, len) || hipMemcpy(d, h.data(), len, hipMemcpyHostToDevice) ||
        hipMalloc(&out, (size_t)blocks * threads * 4) || hipMalloc(&cyc, 8))
        return 1;
    for (int mode = 0; mode < 2; ++mode) {
        (void)hipMemset(cyc, 0, 8);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_simt, dim3(blocks), dim3(threads), 0, 0, d, stream_bytes, nbins, mode, out, cyc);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double lanes = (double)blocks * threads;
        printf("mode %d (%s): %d waves/CU  %.2f Gbins/s chip (%.1f ms)\n", mode,
               mode == 0 ? "ctx bins" : "ctx/bypass divergent", blocks_per_cu * 4, lanes * nbins / (ms * 1e-3) / 1e9,
               ms);
    }
    return 0;
}
