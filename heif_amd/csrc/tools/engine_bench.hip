// engine_bench.hip — single-wave CABAC decision latency (tuning only).
//
// One substream per wave, one wave per SIMD: the latency of one decision bin
// on the dependency chain, which bounds the solo / spread parse of one image
// (its WPP critical path is ~130 k bins).  Variants:
//   0  branch-free VALU decision (parse_lanes.hip dec_s) on wave-uniform
//      values held in VGPRs, state rows by v_readlane, contexts in a VGPR by
//      v_readlane / v_writelane
//   1  the same decision in scalar registers (values made uniform with
//      v_readfirstlane each bin, so the compiler emits SALU)
//   2  scalar, branchy (MPS path first), renormalisation by bits_needed
//   3  variant 1 with the bin value folded into the next context index
//      (sig_coeff_flag-like data dependence)
//   build: make -C heif_amd/csrc engine_bench ; run: build/engine_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../kernels/cabac.hpp"
#include "../kernels/tables.hpp"

extern "C" __device__ int hg_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace {
__constant__ uint8_t c_lps_e[256] = {HG_LPS_TABLE};
__constant__ uint8_t c_trans_e[64] = {HG_TRANS_LPS};

__device__ __forceinline__ uint32_t rl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

template <int V>
__global__ void __launch_bounds__(256) k_eng(const uint32_t *bits, int nbins, uint32_t *out, unsigned long long *cyc) {
    const int lane = threadIdx.x & 63;
    __shared__ uint64_t ltab[64];
    __shared__ uint8_t lctx[256];
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        ltab[t] = (uint64_t)((uint32_t)c_lps_e[t * 4] | ((uint32_t)c_lps_e[t * 4 + 1] << 8) |
                             ((uint32_t)c_lps_e[t * 4 + 2] << 16) | ((uint32_t)c_lps_e[t * 4 + 3] << 24)) |
                  ((uint64_t)((uint32_t)c_trans_e[t] | ((uint32_t)(t < 62 ? t + 1 : t) << 8)) << 32);
    }
    lctx[threadIdx.x] = (uint8_t)((threadIdx.x * 37 + 11) & 0x7f);
    __syncthreads();
    // state rows: rangeTabLps[4] | transLps << 32 | transMps << 40 (lane = pStateIdx)
    const uint32_t tlo = (uint32_t)c_lps_e[lane * 4] | ((uint32_t)c_lps_e[lane * 4 + 1] << 8) |
                         ((uint32_t)c_lps_e[lane * 4 + 2] << 16) | ((uint32_t)c_lps_e[lane * 4 + 3] << 24);
    const uint32_t thi = (uint32_t)c_trans_e[lane] | ((uint32_t)(lane < 62 ? lane + 1 : lane) << 8);
    uint32_t cx = 0x40404040u ^ (uint32_t)(lane * 0x01020304u);  // context bytes, 4 per lane
    const uint32_t *src = bits + (size_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 4096;
    uint32_t win = src[lane];  // 256-byte window, refilled per 64 dwords
    uint32_t rd = 0;
    uint32_t range = 510, value = 0;
    int k = -9;
    uint64_t cur = 0;
    int cn = 0;
    auto pop = [&]() {
        const uint32_t w = rl(win, (int)(rd & 63));
        ++rd;
        return (w >> 24) | ((w >> 8) & 0xff00u) | ((w << 8) & 0xff0000u) | (w << 24);
    };
    auto vfill = [&]() {
        if (cn < 16) {
            cur |= (uint64_t)pop() << (32 - cn);
            cn += 32;
        }
        value = (value << 16) | (uint32_t)(cur >> 48);
        cur <<= 16;
        cn -= 16;
        k += 16;
    };
    vfill();
    vfill();
    uint32_t acc = 0;
    int ci = 5;
    int bits_needed = -8;  // variant 2
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < nbins; ++i) {
        if ((rd & 63) > 56) {  // window refill (rare; not what is measured)
            win = src[(rd + lane) & 4095];
            rd &= ~63u;
        }
        int bin;
        if (V == 2) {
            const uint32_t w = rl(cx, ci >> 2);
            const int sh = (ci & 3) * 8;
            uint32_t s = (w >> sh) & 0xffu, st = s >> 1, mps = s & 1;
            const uint32_t row = rl(tlo, (int)st);
            const uint32_t lps = (row >> (((range >> 6) & 3) * 8)) & 0xffu;
            range -= lps;
            const uint32_t scaled = range << 7;
            if (value < scaled) {
                bin = (int)mps;
                st = st < 62 ? st + 1 : st;
                if (scaled < (256u << 7)) {
                    range = scaled >> 6;
                    value <<= 1;
                    if (++bits_needed == 0) {
                        bits_needed = -8;
                        value |= pop() & 0xffu;
                    }
                }
            } else {
                value -= scaled;
                const int nb = __builtin_clz(lps) - 23;
                value <<= nb;
                range = lps << nb;
                bin = (int)(mps ^ 1u);
                if (st == 0) mps ^= 1u;
                st = rl(thi, (int)st) & 0xffu;
                bits_needed += nb;
                if (bits_needed >= 0) {
                    value |= (pop() & 0xffu) << bits_needed;
                    bits_needed -= 8;
                }
            }
            cx = (uint32_t)hg_writelane((int)((w & ~(0xffu << sh)) | (((st << 1) | mps) << sh)), ci >> 2, (int)cx);
        } else if (V >= 4) {
            // mask arithmetic, no VCC: k <= 22 keeps value < 2^31, so value >= sr is the sign of
            // value - sr; selects are v_bfi_b32 with that mask.  V 4: rows by v_readlane; V 5:
            // rows from LDS (the lanes kernel's per-lane gather); V 6: 5 with the context in LDS
            const int sh = (ci & 3) * 8;
            uint32_t w, s;
            if (V == 6) {
                s = lctx[(ci & 63) + 64 * (threadIdx.x >> 6)];
                w = 0;
            } else {
                w = rl(cx, ci >> 2);
                s = (w >> sh) & 0xffu;
            }
            const uint32_t st = s >> 1, mps = s & 1u;
            uint32_t lo, hi;
            if (V == 4) {
                lo = rl(tlo, (int)st), hi = rl(thi, (int)st);
            } else {
                const uint64_t row = ltab[st];
                lo = (uint32_t)row, hi = (uint32_t)(row >> 32);
            }
            const uint32_t lps = (lo >> ((range >> 3) & 24u)) & 0xffu;
            const uint32_t rm = range - lps;
            const uint32_t sr = rm << k;
            const uint32_t m = (uint32_t)(~((int32_t)(value - sr)) >> 31);  // value >= sr: LPS
            value -= sr & m;
            const uint32_t rn = (m & lps) | (~m & rm);
            const int nb = __builtin_clz(rn) - 23;
            range = rn << nb;
            k -= nb;
            const uint32_t nst = ((m & hi) | (~m & (hi >> 8))) & 0xffu;
            const uint32_t flip = m & ((st - 1u) >> 31);  // LPS in state 0 flips valMps
            const uint32_t ns = (nst << 1) | ((mps ^ flip) & 1u);
            if (V == 6) lctx[(ci & 63) + 64 * (threadIdx.x >> 6)] = (uint8_t)ns;
            else cx = (uint32_t)hg_writelane((int)((w & ~(0xffu << sh)) | (ns << sh)), ci >> 2, (int)cx);
            if (k < 7) vfill();
            bin = (int)((mps ^ m) & 1u);
        } else {
            if (V == 1 || V == 3) {
                range = rfl(range), value = rfl(value), k = (int)rfl((uint32_t)k), ci = (int)rfl((uint32_t)ci);
            }
            const int sh = (ci & 3) * 8;
            const uint32_t w = rl(cx, ci >> 2);
            const uint32_t s = (w >> sh) & 0xffu, st = s >> 1, mps = s & 1u;
            const uint32_t lo = rl(tlo, (int)st), hi = rl(thi, (int)st);
            const uint32_t lps = (lo >> (((range >> 6) & 3u) << 3)) & 0xffu;
            const uint32_t rm = range - lps;
            const uint32_t sr = rm << k;
            const bool isl = value >= sr;
            value -= isl ? sr : 0u;
            const uint32_t rn = isl ? lps : rm;
            const int nb = __builtin_clz(rn) - 23;
            range = rn << nb;
            k -= nb;
            const uint32_t nst = isl ? (hi & 0xffu) : ((hi >> 8) & 0xffu);
            const uint32_t ns = (nst << 1) | (mps ^ ((isl && st == 0) ? 1u : 0u));
            cx = (uint32_t)hg_writelane((int)((w & ~(0xffu << sh)) | (ns << sh)), ci >> 2, (int)cx);
            if (k < 8) vfill();
            bin = (int)(mps ^ (isl ? 1u : 0u));
        }
        acc += (uint32_t)bin;
        ci = V == 3 ? ((ci + 1 + bin) & 63) : ((ci + 3) & 63);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc + range + (uint32_t)k;
        atomicAdd(cyc, (unsigned long long)(t1 - t0));
    }
}
}  // namespace

int main() {
    const int nbins = 100000, blocks = 256;  // one wave per SIMD
    std::vector<uint32_t> h((size_t)blocks * 4 * 4096);
    uint64_t x = 88172645463325252ull;
    for (auto &b : h) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = (uint32_t)x;
    }
    uint32_t *d, *out;
    unsigned long long *cyc;
    hipMalloc(&d, h.size() * 4);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&out, blocks * 16);
    hipMalloc(&cyc, 8);
    void (*ks[7])(const uint32_t *, int, uint32_t *, unsigned long long *) = {k_eng<0>, k_eng<1>, k_eng<2>, k_eng<3>,
                                                                             k_eng<4>, k_eng<5>, k_eng<6>};
    const char *names[7] = {"VALU branch-free (solo dec_s)", "SALU branch-free", "SALU branchy, byte renorm",
                            "SALU branch-free, bin-dependent ctx", "VALU masks+bfi, readlane rows",
                            "VALU masks+bfi, LDS rows", "VALU masks+bfi, LDS rows + LDS ctx"};
    setvbuf(stdout, nullptr, _IONBF, 0);
    for (int v = 0; v < 7; ++v) {
        hipMemset(cyc, 0, 8);
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, d, nbins, out, cyc);
        hipDeviceSynchronize();
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("variant %d %-38s %.1f cycles/bin (one wave per SIMD)\n", v, names[v], (double)c / (blocks * 4.0) / nbins);
    }
    return 0;
}
