// common.hpp — shared internals of libccrdt (host + device).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <initializer_list>
#include <string>

#include "../../include/ccrdt.h"

namespace ccrdt {

void set_error(const std::string& msg);

#define CCRDT_HIP(call)                                                        \
  do {                                                                         \
    hipError_t _e = (call);                                                    \
    if (_e != hipSuccess) {                                                    \
      ::ccrdt::set_error(std::string(#call) + ": " + hipGetErrorString(_e));   \
      return CCRDT_EDEVICE;                                                    \
    }                                                                          \
  } while (0)

#define CCRDT_TRY(call)          \
  do {                           \
    int _rc = (call);            \
    if (_rc != CCRDT_OK) return _rc; \
  } while (0)

// Grow-only device buffer.
struct DevBuf {
  void* p = nullptr;
  uint64_t bytes = 0;
  int ensure(uint64_t need) {
    if (need <= bytes && p) return CCRDT_OK;
    if (p) {
      CCRDT_HIP(hipFree(p));
      p = nullptr;
      bytes = 0;
    }
    uint64_t b = need < 256 ? 256 : need;
    CCRDT_HIP(hipMalloc(&p, b));
    bytes = b;
    return CCRDT_OK;
  }
  // Growth with headroom for state that grows batch after batch (the
  // resident topk_rmv sides): a buffer that must grow is re-allocated at
  // twice the request, so a steady stream re-allocates every few batches
  // instead of at each (a re-allocation of GBs costs milliseconds).
  // When the doubled size does not fit on the device, the exact need is tried.
  int ensure_grow(uint64_t need) {
    if (need <= bytes && p) return CCRDT_OK;
    if (!p) return ensure(need);
    CCRDT_HIP(hipFree(p));
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, 2 * need) == hipSuccess) {
      bytes = 2 * need;
      return CCRDT_OK;
    }
    p = nullptr;
    (void)hipGetLastError();  // (the failed allocation's error is not sticky)
    return ensure(need);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// ------------------------------------------------------------ wave helpers
// One wavefront = 64 lanes on CDNA4.  These helpers move wave-uniform values
// between lanes and SGPRs.

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Bounds-checked loads through a buffer descriptor over [base, base + bytes):
// a lane whose byte offset lies past the range reads 0 -- no branch around
// the load, no fault -- so a run of conditional loads issues back to back.
// The descriptor's inputs are made provably wave-uniform (readfirstlane):
// the caller's base and size must be the same on every lane.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bsrc(const void* base, uint32_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr uint32_t BOOB = 0x7FFFFFF0u;  // an open-ended range, and the offset that reads past it
__device__ __forceinline__ int64_t bld64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  return (int64_t)(((uint64_t)v[1] << 32) | v[0]);
}
__device__ __forceinline__ uint32_t bld32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}
__device__ __forceinline__ uint32_t bld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b16(r, (int)off, 0, 0);
}
__device__ __forceinline__ uint32_t bld8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b8(r, (int)off, 0, 0);
}

__device__ __forceinline__ uint32_t rl32(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ int64_t rl64(int64_t v, int lane) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// Write v into one lane (wave-uniform lane index): v_cmp + v_cndmask.
__device__ __forceinline__ uint32_t wl32(uint32_t old, int lane, uint32_t v) {
  return (int)(threadIdx.x & 63) == lane ? v : old;
}
__device__ __forceinline__ int64_t wl64(int64_t old, int lane, int64_t v) {
  return (int)(threadIdx.x & 63) == lane ? v : old;
}
// Per-lane gather from another lane (ds_bpermute crossbar).
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ int64_t shfl64(int64_t v, int src) {
  uint32_t lo = shfl32((uint32_t)v, src);
  uint32_t hi = shfl32((uint32_t)((uint64_t)v >> 32), src);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
// Number of set bits of m below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
// Exclusive prefix sum over the 64 lanes; `total` = wave sum.
__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t v, uint32_t& total) {
  const int lane = lane_id();
  uint32_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = shfl32(inc, lane >= off ? lane - off : lane);
    if (lane >= off) inc += o;
  }
  total = rl32(inc, 63);
  return inc - v;
}
// Inclusive prefix sum over the 64 lanes in 6 DPP adds (no LDS crossbar):
// row_shr 1/2/4/8 scan each 16-lane row, row_bcast:15/31 carry the row
// totals into the rows above.  Lanes a DPP source cannot reach add `old` = 0.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}
// Wave minimum of an int64 in 6 DPP steps (same row_shr / row_bcast pattern
// as wave_incl_scan_dpp); lanes without a DPP source see INT64_MAX.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int64_t dpp_min_step_i64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)(uint32_t)v, CTRL,
                                                            ROWMASK, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(
      (int)0x7FFFFFFF, (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROWMASK, 0xf, false);
  const int64_t o = (int64_t)(((uint64_t)hi << 32) | lo);
  return o < v ? o : v;
}
__device__ __forceinline__ int64_t wave_min_i64_dpp(int64_t v) {
  v = dpp_min_step_i64<0x111, 0xf>(v);
  v = dpp_min_step_i64<0x112, 0xf>(v);
  v = dpp_min_step_i64<0x114, 0xf>(v);
  v = dpp_min_step_i64<0x118, 0xf>(v);
  v = dpp_min_step_i64<0x142, 0xa>(v);
  v = dpp_min_step_i64<0x143, 0xc>(v);
  return rl64(v, 63);
}
// Wave maximum of a uint32 (DPP, identity 0), wave-uniform result.
__device__ __forceinline__ uint32_t wave_max_u32_dpp(uint32_t v) {
  uint32_t o;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v = o > v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  v = o > v ? o : v;
  return rl32(v, 63);
}
// Wave minimum of a uint32 (DPP, identity 0xFFFFFFFF), wave-uniform result.
__device__ __forceinline__ uint32_t wave_min_u32_dpp(uint32_t v) {
  uint32_t o;
  o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xf, 0xf, false);
  v = o < v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xf, 0xf, false);
  v = o < v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xf, 0xf, false);
  v = o < v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xf, 0xf, false);
  v = o < v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xa, 0xf, false);
  v = o < v ? o : v;
  o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xc, 0xf, false);
  v = o < v ? o : v;
  return rl32(v, 63);
}
// Exclusive DPP scan; `total` = wave sum (wave-uniform).
__device__ __forceinline__ uint32_t wave_excl_scan_dpp(uint32_t v, uint32_t& total) {
  const uint32_t inc = wave_incl_scan_dpp(v);
  total = rl32(inc, 63);
  return inc - v;
}
// A kernel's FIRST parameter (a struct of type T, at kernarg offset 0) read
// from the kernarg segment through a pointer the compiler cannot see
// through, so each use is a scalar load at the point of use instead of a
// value held in SGPRs across the kernel (where it spills to VGPR lanes and
// returns by v_readlane).  Only in kernels whose first parameter is a T.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* kernarg_as() {
  const __attribute__((address_space(4))) T* p =
      (const __attribute__((address_space(4))) T*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// Orders one wavefront's LDS accesses across lanes without a workgroup
// barrier.  The LDS executes (and returns) a wave's DS instructions in issue
// order, so a later DS instruction of the wave sees every earlier one's
// effect; all this has to stop is the compiler moving accesses across the
// point (it reasons per lane and cannot see that lanes share addresses).
// No s_waitcnt: a wavefront-scope fence would wait for every outstanding DS
// op (a full LDS round trip) at each such point.  -DCCRDT_LDS_FENCE builds
// the fenced form instead.
__device__ __forceinline__ void wave_lds_sync() {
#ifdef CCRDT_LDS_FENCE
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#else
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// Wave maximum of an int64 (DPP, identity INT64_MIN), wave-uniform result.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int64_t dpp_max_step_i64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROWMASK, 0xf,
                                                            false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(
      (int)0x80000000, (int)(uint32_t)((uint64_t)v >> 32), CTRL, ROWMASK, 0xf, false);
  const int64_t o = (int64_t)(((uint64_t)hi << 32) | lo);
  return o > v ? o : v;
}
__device__ __forceinline__ int64_t wave_max_i64_dpp(int64_t v) {
  v = dpp_max_step_i64<0x111, 0xf>(v);
  v = dpp_max_step_i64<0x112, 0xf>(v);
  v = dpp_max_step_i64<0x114, 0xf>(v);
  v = dpp_max_step_i64<0x118, 0xf>(v);
  v = dpp_max_step_i64<0x142, 0xa>(v);
  v = dpp_max_step_i64<0x143, 0xc>(v);
  return rl64(v, 63);
}

// Wave min / max over all 64 lanes (every lane active), wave-uniform result:
// six DPP steps, no LDS-crossbar round trips on the reduction's latency chain.
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) { return wave_min_i64_dpp(v); }
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) { return wave_max_i64_dpp(v); }

// A kernel's first launch in a process sets up its function object (about
// 0.1 ms each, measured: tools/first_use.py); hipFuncGetAttributes does the
// same set-up, so an engine does it for its kernels at creation instead of
// inside its first batch.
template <typename... Kern>
inline void preload_kernels(Kern... k) {
  hipFuncAttributes at;
  (void)std::initializer_list<int>{((void)hipFuncGetAttributes(&at, reinterpret_cast<const void*>(k)), 0)...};
  (void)hipGetLastError();  // (a failure here only means the first launch does the set-up)
}

}  // namespace ccrdt
