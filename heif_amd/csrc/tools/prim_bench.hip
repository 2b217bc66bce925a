// prim_bench.hip — dependent-chain latency of the primitives a single-wave
// CABAC engine is built from (tuning only).  One wave per SIMD, s_memtime
// around 1000 iterations of an 8-deep dependent chain; prints cycles per op.
//   build: make -C heif_amd/csrc prim_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

namespace {
constexpr int kIters = 1000;

template <int V>
__global__ void __launch_bounds__(256) k_prim(const uint32_t *tab, uint32_t *out, unsigned long long *cyc) {
    __shared__ uint32_t lds[256];
    const int lane = threadIdx.x & 63;
    lds[threadIdx.x] = (threadIdx.x * 7 + 1) & 63;
    __syncthreads();
    uint32_t v = (uint32_t)(lane * 7 + 1) & 63;  // lane i holds a next index
    uint32_t s = 3;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
        if (V == 0) {  // SALU dependent add
            asm volatile("s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n"
                         "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 1"
                         : "+s"(s));
        } else if (V == 1) {  // VALU dependent add
            asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n"
                         "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1"
                         : "+v"(v));
        } else if (V == 2) {  // v_readlane whose lane index is the previous result (table walk in a VGPR)
            for (int k = 0; k < 8; ++k) s = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)(s & 63));
        } else if (V == 3) {  // LDS load at the previous result (uniform address)
            for (int k = 0; k < 8; ++k) s = __builtin_amdgcn_readfirstlane(lds[s & 63]);
        } else if (V == 4) {  // scalar-cache load at the previous result
            for (int k = 0; k < 8; ++k) s = __builtin_amdgcn_readfirstlane(tab[s & 63]) ;
        } else if (V == 5) {  // v_readlane then SALU use then VALU use (VALU -> SGPR -> VALU round trip)
            for (int k = 0; k < 8; ++k) {
                s = (uint32_t)__builtin_amdgcn_readlane((int)v, 5) + s;
                v += s;
            }
        } else if (V == 6) {  // VALU compare -> SCC/VCC -> select chain (branch-free decision shape)
            for (int k = 0; k < 8; ++k) {
                const bool c = v >= (s & 127);
                v = c ? v - 13 : v + 29;
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s + v;
        atomicAdd(cyc, (unsigned long long)(t1 - t0));
    }
}
}  // namespace

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int blocks = 256;
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    uint32_t *tab, *out;
    unsigned long long *cyc;
    uint32_t h[64];
    for (int i = 0; i < 64; ++i) h[i] = (i * 13 + 5) & 63;
    (void)hipMalloc(&tab, 256);
    (void)hipMemcpy(tab, h, 256, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, blocks * 16);
    (void)hipMalloc(&cyc, 8);
    void (*ks[7])(const uint32_t *, uint32_t *, unsigned long long *) = {k_prim<0>, k_prim<1>, k_prim<2>, k_prim<3>,
                                                                        k_prim<4>, k_prim<5>, k_prim<6>};
    const char *names[7] = {"s_add chain", "v_add chain", "v_readlane index chain", "LDS load chain (uniform)",
                            "global load chain (uniform, cached)", "v_readlane->SALU->VALU round trip",
                            "VALU compare+select chain"};
    for (int v = 0; v < 7; ++v) {
        if (only >= 0 && v != only) continue;
        printf("%d ", v);
        (void)hipMemset(cyc, 0, 8);
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, tab, out, cyc);
        (void)hipDeviceSynchronize();
        unsigned long long c = 0;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-40s %.1f cycles/op\n", names[v], (double)c / (blocks * 4.0) / (kIters * 8.0));
    }
    return 0;
}
