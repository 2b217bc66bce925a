// wave.hpp — the few wave-level primitives the decode kernels use, with a
// host-emulation variant.
//
// On gfx950 (default) these are the real 64-lane wave64 intrinsics.  With
// HG_HOST_EMU defined the same kernel sources compile as plain C++ for the
// host: each wave runs as one host thread with a single lane (kWave = 1, so
// every `for (k = lane; k < n; k += kWave)` loop covers all of its work), LDS
// becomes a per-block static buffer, and block barriers / LDS atomics map to
// std::atomic.  That build exists only for tests (AddressSanitizer runs and
// CPU-side parity of the kernels' intermediate records against the oracle);
// it is never loaded by the product path.
#pragma once
#include <stdint.h>

#if defined(HG_HOST_EMU)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __constant__
#define __launch_bounds__(...)
#define HG_SHARED static thread_local
#define HG_BLOCK_SHARED static

namespace hg {
constexpr int kWave = 1;
struct EmuDim3 {
    unsigned x = 0, y = 0, z = 0;
};
struct EmuCtx {
    EmuDim3 bidx, tidx, bdim, gdim;
    unsigned char *smem;  // exact-size dynamic LDS of the current block (heap, ASan-checked)
    std::atomic<int> *bar_count;
    std::atomic<int> *bar_gen;
    int bar_n;
};
extern thread_local EmuCtx g_emu;
inline void emu_syncthreads() {
    int gen = g_emu.bar_gen->load();
    if (g_emu.bar_count->fetch_add(1) + 1 == g_emu.bar_n) {
        g_emu.bar_count->store(0);
        g_emu.bar_gen->fetch_add(1);
    } else {
        while (g_emu.bar_gen->load() == gen) std::this_thread::yield();
    }
}
}  // namespace hg
#define blockIdx (::hg::g_emu.bidx)
#define threadIdx (::hg::g_emu.tidx)
#define blockDim (::hg::g_emu.bdim)
#define gridDim (::hg::g_emu.gdim)
#define __syncthreads() ::hg::emu_syncthreads()
#define HG_UNI(v) (v)
#define HG_GAS
#define HG_FENCE_ACQ() std::atomic_thread_fence(std::memory_order_acquire)
#define HG_FENCE_REL() std::atomic_thread_fence(std::memory_order_release)
#define HG_ACQ_AGENT() std::atomic_thread_fence(std::memory_order_acquire)
#define HG_REL_AGENT() std::atomic_thread_fence(std::memory_order_release)
#define HG_WAVE_SYNC() ((void)0)
#define HG_SLEEP() std::this_thread::yield()
template <class T>
inline T hg_atomic_load(T *p) {
    return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}
// a word another kernel of the same decode writes (agent scope on the GPU)
inline uint32_t hg_load_agent(const uint32_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
// a clock in 10 ns ticks (the GPU's 100 MHz real-time counter)
inline uint64_t hg_clock_10ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count() / 10;
}
template <class T>
inline void hg_atomic_store(T *p, T v) {
    __atomic_store_n(p, v, __ATOMIC_RELEASE);
}
inline void atomicOr(uint32_t *p, uint32_t v) { __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
inline void atomicMax(int32_t *p, int32_t v) {
    int32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
}
using std::max;
using std::min;
#else
#include <hip/hip_runtime.h>
#define HG_SHARED __shared__
#define HG_BLOCK_SHARED __shared__
namespace hg {
constexpr int kWave = 64;
}
#define HG_UNI(v) __builtin_amdgcn_readfirstlane(v)
// global address space (a pointer type qualifier; host emulation: none)
#if defined(__HIP_DEVICE_COMPILE__)
#define HG_GAS __attribute__((address_space(1)))
#else
#define HG_GAS
#endif
#define HG_FENCE_ACQ() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup")
#define HG_FENCE_REL() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup")
// Cross-CU hand-offs (another workgroup, possibly on another XCD: MI355X_MICROARCH.md
// "inter-workgroup visibility").  Consumer: after the relaxed poll has matched,
// an agent acquire (s_waitcnt vmcnt(0); buffer_inv sc1: this CU's L1 dropped)
// before the handed-off bytes are read.  Producer: an agent release (buffer_wbl2
// sc1; s_waitcnt vmcnt(0)), then the explicit wait the guide prescribes (the
// compiler may drop its own after the write-back), then the relaxed flag store.
#if defined(HG_HANDOFF_RELAXED)  // A/B only: the r04 forms (vmcnt(0) + sc1 flag; no acquire)
#define HG_ACQ_AGENT() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup")
#define HG_REL_AGENT() __builtin_amdgcn_s_waitcnt(0x0f70)
#else
#define HG_ACQ_AGENT() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent")
#define HG_REL_AGENT()                                  \
    do {                                                \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  \
    } while (0)
#endif
// Orders one wave's own LDS traffic across lanes (write by lane i, read by
// lane j).  A wave's LDS instructions execute in order, so wavefront scope is
// enough; workgroup scope would also drain the wave's outstanding global
// stores (s_waitcnt vmcnt(0)) at every call.
#define HG_WAVE_SYNC()                                       \
    do {                                                     \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                     \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
    } while (0)
#define HG_SLEEP() __builtin_amdgcn_s_sleep(2)
// Issue priority of the parse stream's kernels (k_rbsp, k_parse_lanes,
// k_parse_solo): s_setprio HG_PARSE_SETPRIO, 0 turns it off for all of them
// (r04 A/B: 128 images 83.5-83.8 vs 84.4 ms per step, one image 27.8 vs
// 28.05 ms)
#if !defined(HG_PARSE_SETPRIO)
#define HG_PARSE_SETPRIO 3
#endif
template <class T>
__device__ __forceinline__ T hg_atomic_load(T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a word another kernel of the same decode writes (agent scope: coherent across XCDs)
__device__ __forceinline__ uint32_t hg_load_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a clock in 10 ns ticks (s_memrealtime: the 100 MHz real-time counter, one for the whole chip)
__device__ __forceinline__ uint64_t hg_clock_10ns() { return __builtin_amdgcn_s_memrealtime(); }
template <class T>
__device__ __forceinline__ void hg_atomic_store(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
#endif
