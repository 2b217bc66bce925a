// Probe of the gfx950 int8 MFMA operand maps assumed by the transform
// (exact integer data, asymmetric A and B): prints OK / the first mismatch.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe/mfma_i8_probe.cpp -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 32x32x32: lane l (r = l & 31, h = l >> 5) holds A[r][16h + j] and B[16h + j][r] (j < 16);
// D register i: row (i & 3) + 8 (i >> 2) + 4h, column r
__global__ void k32(const int8_t *A, const int8_t *B, int *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[r * 32 + 16 * h + j];
        b[j] = B[(16 * h + j) * 32 + r];
    }
    v4i fa, fb;
    __builtin_memcpy(&fa, a, 16);
    __builtin_memcpy(&fb, b, 16);
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}
// 16x16x64: lane l (r = l & 15, g = l >> 4) holds A[r][16g + j] and B[16g + j][r];
// D register i: row 4g + i, column r
__global__ void k16(const int8_t *A, const int8_t *B, int *D) {
    const int l = threadIdx.x, r = l & 15, g = l >> 4;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[r * 64 + 16 * g + j];
        b[j] = B[(16 * g + j) * 16 + r];
    }
    v4i fa, fb;
    __builtin_memcpy(&fa, a, 16);
    __builtin_memcpy(&fb, b, 16);
    v4i c = {};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, fb, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = c[i];
}

static int check(const char *name, int M, int N, int K, void (*kern)(const int8_t *, const int8_t *, int *)) {
    std::vector<int8_t> A(M * K), B(K * N);
    for (int i = 0; i < M * K; ++i) A[i] = (int8_t)((i * 37 + 11) % 251 - 125);
    for (int i = 0; i < K * N; ++i) B[i] = (int8_t)((i * 53 + 7) % 241 - 120);
    int8_t *dA, *dB;
    int *dD;
    hipMalloc(&dA, A.size());
    hipMalloc(&dB, B.size());
    hipMalloc(&dD, M * N * 4);
    hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
    hipMemset(dD, 0, M * N * 4);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    std::vector<int> D(M * N);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < M && !bad; ++i)
        for (int j = 0; j < N && !bad; ++j) {
            long s = 0;
            for (int k = 0; k < K; ++k) s += (long)A[i * K + k] * B[k * N + j];
            if (s != D[i * N + j]) {
                printf("%s MISMATCH at [%d][%d]: %ld vs %d\n", name, i, j, s, D[i * N + j]);
                bad = 1;
            }
        }
    if (!bad) printf("%s OK\n", name);
    hipFree(dA);
    hipFree(dB);
    hipFree(dD);
    return bad;
}

int main() {
    int bad = check("mfma_i32_32x32x32_i8", 32, 32, 32, k32);
    bad |= check("mfma_i32_16x16x64_i8", 16, 16, 64, k16);
    return bad;
}
