// staging.cpp — host -> device upload of pageable caller memory through a
// pinned staging ring (the host-array entry points, e.g. ccrdt_trmv_apply).
//
// A plain hipMemcpyAsync from pageable memory goes through the runtime's
// own bounce buffers one piece at a time (~1-2 GB/s for a 3 GB batch).  Here
// STAGE_THREADS host threads each own one pinned slot of STAGE_CHUNK bytes:
// thread t copies chunks t, t+T, ... of the source into its slot (memcpy,
// the threads run in parallel) and queues the slot's DMA on the engine
// stream, waiting for the slot's previous DMA (its event) before refilling
// it.  The kernels the caller launches afterwards on the same stream run
// after every DMA; the caller's memory is no longer read once this returns.
#include <immintrin.h>
#include <sched.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "engine.hpp"

namespace ccrdt {

int launch_widen_i64(int64_t* dst, const int32_t* src, const int64_t* base, const uint8_t* kind,
                     uint64_t n, uint64_t chunk, hipStream_t st);
int launch_widen_ops(int64_t* id, int64_t* score, int64_t* ts, const int32_t* src, const int64_t* base,
                     const uint8_t* kind, uint64_t n, uint64_t chunk, hipStream_t st);

namespace {
constexpr int STAGE_THREADS = 16;                       // (at most; see stage_threads)
constexpr uint64_t STAGE_CHUNK = 16ull << 20;          // bytes per slot
constexpr uint64_t STAGE_DIRECT = 4ull << 20;           // below: one plain copy
constexpr uint64_t NARROW_CHUNK = STAGE_CHUNK / 16;     // int32 elements per chunk (a quarter slot: the
                                                        // threads stay busy to the column's end)
constexpr uint64_t NARROW_MAX_CHUNKS = 4096;            // (4 Gi elements)
constexpr uint64_t OPS_CHUNK = 1ull << 20;              // ops per slot in h2d_trmv_ops (14 B each)
static_assert(OPS_CHUNK * 14 <= STAGE_CHUNK, "an ops chunk fits one slot");
}  // namespace

// Staging threads: the CPUs this process may use (affinity), at most
// STAGE_THREADS (each owns a pinned slot).
static int stage_threads() {
  static const int n = [] {
    cpu_set_t cs;
    int c = 8;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) c = CPU_COUNT(&cs);
    return std::max(1, std::min(STAGE_THREADS, c));
  }();
  return n;
}

// One chunk of an int64 column narrowed to int32 (see h2d_staged_i64): a
// branch-free loop the compiler vectorizes; false if a value leaves int32.
__attribute__((target("avx2"))) static bool narrow_chunk_avx2(const int64_t* src, const uint8_t* kind,
                                                               int32_t* out, uint64_t len, int64_t base) {
  uint64_t bad = 0;
  if (!kind) {
    for (uint64_t i = 0; i < len; ++i) {
      const int64_t v = (int64_t)((uint64_t)src[i] - (uint64_t)base);  // (modulo 2^64: exact round trip)
      out[i] = (int32_t)v;
      bad |= (uint64_t)((v >> 31) ^ (v >> 63));
    }
  } else {
    for (uint64_t i = 0; i < len; ++i) {
      const int64_t v = (int64_t)((uint64_t)src[i] - (uint64_t)(kind[i] < 2 ? base : 0));
      out[i] = (int32_t)v;
      bad |= (uint64_t)((v >> 31) ^ (v >> 63));
    }
  }
  return bad == 0;
}
static bool narrow_chunk_plain(const int64_t* src, const uint8_t* kind, int32_t* out, uint64_t len, int64_t base) {
  uint64_t bad = 0;
  for (uint64_t i = 0; i < len; ++i) {
    const int64_t v = (int64_t)((uint64_t)src[i] - (uint64_t)((!kind || kind[i] < 2) ? base : 0));
    out[i] = (int32_t)v;
    bad |= (uint64_t)((v >> 31) ^ (v >> 63));
  }
  return bad == 0;
}

// memset on the staging threads (a host output buffer of n_ops bytes: its
// first touch is page faults, which the threads take in parallel)
void host_fill(void* dst, int v, uint64_t bytes) {
  constexpr uint64_t PART = 8ull << 20;
  const uint64_t parts = (bytes + PART - 1) / PART;
  const int T = (int)std::min<uint64_t>((uint64_t)stage_threads(), parts);
  if (T <= 1) {
    memset(dst, v, bytes);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (int t = 0; t < T; ++t)
    th.emplace_back([=] {
      for (uint64_t c = (uint64_t)t; c < parts; c += (uint64_t)T) {
        const uint64_t off = c * PART;
        memset(static_cast<char*>(dst) + off, v, std::min<uint64_t>(PART, bytes - off));
      }
    });
  for (std::thread& x : th) x.join();
}

static int stage_init(Engine& E) {
  if (E.pin_n) return CCRDT_OK;
  for (int t = 0; t < stage_threads(); ++t) {
    CCRDT_HIP(hipHostMalloc(&E.pin[t], STAGE_CHUNK, hipHostMallocDefault));
    CCRDT_HIP(hipEventCreateWithFlags(&E.pin_ev[t], hipEventDisableTiming));
    CCRDT_HIP(hipEventRecord(E.pin_ev[t], E.stream));  // "slot free"
    E.pin_n = t + 1;
  }
  return CCRDT_OK;
}

static int narrow_init(Engine& E) {
  if (E.pin_base) return CCRDT_OK;
  CCRDT_HIP(hipHostMalloc(&E.pin_base, NARROW_MAX_CHUNKS * 8 * 3, hipHostMallocDefault));
  for (hipEvent_t& v : E.pin_bev) {
    CCRDT_HIP(hipEventCreateWithFlags(&v, hipEventDisableTiming));
    CCRDT_HIP(hipEventRecord(v, E.stream));
  }
  return CCRDT_OK;
}

void stage_release(Engine& E) {
  if (E.pin_base) (void)hipHostFree(E.pin_base);
  E.pin_base = nullptr;
  for (hipEvent_t& v : E.pin_bev) {
    if (v) (void)hipEventDestroy(v);
    v = nullptr;
  }
  for (int t = 0; t < E.pin_n; ++t) {
    if (E.pin[t]) (void)hipHostFree(E.pin[t]);
    if (E.pin_ev[t]) (void)hipEventDestroy(E.pin_ev[t]);
    E.pin[t] = nullptr;
    E.pin_ev[t] = nullptr;
  }
  E.pin_n = 0;
}

int h2d_staged(Engine& E, void* dst, const void* src, uint64_t bytes) {
  if (!bytes) return CCRDT_OK;
  if (bytes < STAGE_DIRECT) {
    CCRDT_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, E.stream));
    return CCRDT_OK;
  }
  CCRDT_TRY(stage_init(E));
  const uint64_t n_chunks = (bytes + STAGE_CHUNK - 1) / STAGE_CHUNK;
  const int T = (int)std::min<uint64_t>(E.pin_n, n_chunks);
  std::vector<int> rc(T, CCRDT_OK);
  std::vector<std::thread> th;
  th.reserve(T);
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      (void)hipSetDevice(E.device);
      for (uint64_t c = (uint64_t)t; c < n_chunks; c += (uint64_t)T) {
        const uint64_t off = c * STAGE_CHUNK;
        const uint64_t len = std::min<uint64_t>(STAGE_CHUNK, bytes - off);
        // the slot's previous DMA must have read it before it is refilled
        if (hipEventSynchronize(E.pin_ev[t]) != hipSuccess) {
          rc[t] = CCRDT_EDEVICE;
          return;
        }
        memcpy(E.pin[t], static_cast<const char*>(src) + off, len);
        if (hipMemcpyAsync(static_cast<char*>(dst) + off, E.pin[t], len, hipMemcpyHostToDevice, E.stream) !=
                hipSuccess ||
            hipEventRecord(E.pin_ev[t], E.stream) != hipSuccess) {
          rc[t] = CCRDT_EDEVICE;
          return;
        }
      }
    });
  for (std::thread& x : th) x.join();
  for (int t = 0; t < T; ++t)
    if (rc[t] != CCRDT_OK) {
      set_error("h2d_staged: staging copy failed");
      return rc[t];
    }
  return CCRDT_OK;
}

}  // namespace ccrdt

namespace ccrdt {

// An int64 column crosses PCIe as int32: the staging threads convert each
// chunk while they copy it into their pinned slot, a device kernel widens it
// into `dst`.  kind == nullptr: every value travels as it is (Ids, Scores),
// or, with `based` (the removal clocks), as value - base, base = the chunk's
// first value.  kind != nullptr (the Ts column, whose rmv entries are
// clock-row indices): a chunk's adds travel as Ts - base, base = the chunk's
// first add Ts, and its rmv entries as they are.  A value outside int32 anywhere sends
// the whole column wide (h2d_staged) instead; the result is the same.
// `slot` (0..2) picks the chunk-base region of the pinned base buffer, so
// three columns can be in flight on the stream at once.
int h2d_staged_i64(Engine& E, int64_t* dst, const int64_t* src, uint64_t n, const uint8_t* kind,
                   const uint8_t* kind_dev, int slot, DevBuf& scratch, DevBuf& dbase, bool based) {
  if (!n) return CCRDT_OK;
  const uint64_t n_chunks = (n + NARROW_CHUNK - 1) / NARROW_CHUNK;
  if (n < STAGE_DIRECT / 4 || n_chunks > NARROW_MAX_CHUNKS) return h2d_staged(E, dst, src, n * 8);
  CCRDT_TRY(stage_init(E));
  CCRDT_TRY(narrow_init(E));
  CCRDT_TRY(scratch.ensure(n * 4));
  CCRDT_TRY(dbase.ensure(n_chunks * 8));
  int64_t* bases = reinterpret_cast<int64_t*>(E.pin_base) + slot * NARROW_MAX_CHUNKS;
  CCRDT_HIP(hipEventSynchronize(E.pin_bev[slot]));  // the region's previous DMA has read it
  const int T = (int)std::min<uint64_t>(E.pin_n, n_chunks);
  static const bool avx2 = __builtin_cpu_supports("avx2");
  std::vector<int> rc(T, CCRDT_OK);
  std::vector<char> wide(T, 0);
  std::vector<std::thread> th;
  th.reserve(T);
  int32_t* d32 = scratch.as<int32_t>();
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      (void)hipSetDevice(E.device);
      for (uint64_t c = (uint64_t)t; c < n_chunks; c += (uint64_t)T) {
        const uint64_t i0 = c * NARROW_CHUNK;
        const uint64_t len = std::min<uint64_t>(NARROW_CHUNK, n - i0);
        if (hipEventSynchronize(E.pin_ev[t]) != hipSuccess) {
          rc[t] = CCRDT_EDEVICE;
          return;
        }
        int64_t base = based ? src[i0] : 0;
        if (kind)
          for (uint64_t i = i0; i < i0 + len; ++i)
            if (kind[i] < 2) {
              base = src[i];
              break;
            }
        bases[c] = base;
        int32_t* out = static_cast<int32_t*>(E.pin[t]);
        const bool ok = avx2 ? narrow_chunk_avx2(src + i0, kind ? kind + i0 : nullptr, out, len, base)
                             : narrow_chunk_plain(src + i0, kind ? kind + i0 : nullptr, out, len, base);
        if (!ok) {
          wide[t] = 1;
          return;
        }
        if (hipMemcpyAsync(d32 + i0, out, len * 4, hipMemcpyHostToDevice, E.stream) != hipSuccess ||
            hipEventRecord(E.pin_ev[t], E.stream) != hipSuccess) {
          rc[t] = CCRDT_EDEVICE;
          return;
        }
      }
    });
  for (std::thread& x : th) x.join();
  bool any_wide = false;
  for (int t = 0; t < T; ++t) {
    if (rc[t] != CCRDT_OK) {
      set_error("h2d_staged_i64: staging copy failed");
      return rc[t];
    }
    any_wide |= wide[t] != 0;
  }
  if (any_wide) return h2d_staged(E, dst, src, n * 8);
  CCRDT_HIP(hipMemcpyAsync(dbase.p, bases, n_chunks * 8, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipEventRecord(E.pin_bev[slot], E.stream));
  return launch_widen_i64(dst, d32, dbase.as<int64_t>(), kind ? kind_dev : nullptr, n, NARROW_CHUNK, E.stream);
}

// narrow_chunk_avx2 with non-temporal stores (the pinned slot is only read by
// the DMA engine: no read-for-ownership of its lines, no cache pollution).
// `out` 32-byte aligned.  False if a value leaves int32.
__attribute__((target("avx2"))) static bool narrow_stream_avx2(const int64_t* src, const uint8_t* kind, int32_t* out,
                                                                uint64_t len, int64_t base) {
  const __m256i lo = _mm256_setr_epi32(0, 2, 4, 6, 0, 2, 4, 6);
  const __m256i vb = _mm256_set1_epi64x(base), two = _mm256_set1_epi64x(2);
  __m256i bad = _mm256_setzero_si256();
  uint64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 4));
    if (kind) {  // adds (kind < 2) relative to the chunk base
      const __m128i k8 = _mm_loadl_epi64(reinterpret_cast<const __m128i*>(kind + i));
      const __m256i ka = _mm256_cvtepu8_epi64(k8), kb = _mm256_cvtepu8_epi64(_mm_srli_si128(k8, 4));
      a = _mm256_sub_epi64(a, _mm256_and_si256(vb, _mm256_cmpgt_epi64(two, ka)));
      b = _mm256_sub_epi64(b, _mm256_and_si256(vb, _mm256_cmpgt_epi64(two, kb)));
    } else {  // every value relative to the base (0: as it is)
      a = _mm256_sub_epi64(a, vb);
      b = _mm256_sub_epi64(b, vb);
    }
    const __m128i na = _mm256_castsi256_si128(_mm256_permutevar8x32_epi32(a, lo));
    const __m128i nb = _mm256_castsi256_si128(_mm256_permutevar8x32_epi32(b, lo));
    bad = _mm256_or_si256(bad, _mm256_xor_si256(a, _mm256_cvtepi32_epi64(na)));
    bad = _mm256_or_si256(bad, _mm256_xor_si256(b, _mm256_cvtepi32_epi64(nb)));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(out + i), _mm256_inserti128_si256(_mm256_castsi128_si256(na), nb, 1));
  }
  const bool ok = _mm256_testz_si256(bad, bad) != 0;
  return narrow_chunk_avx2(src + i, kind ? kind + i : nullptr, out + i, len - i, base) && ok;
}

// The host batch of ccrdt_trmv_apply in one pass: each chunk of OPS_CHUNK
// ops is staged by one thread into its pinned slot as [Id int32 | Score int32
// | Ts int32 | Kind | DcId] (Ts of adds relative to the chunk's first add Ts,
// rmv entries -- clock-row indices -- as they are) and crosses PCIe as five
// DMAs; one device kernel widens the three int32 columns.  The caller's
// columns are read once, by all threads at once, with no barrier between
// columns.  CCRDT_ERANGE (nothing of the result written yet): a value leaves
// int32 -- the caller uploads column by column instead (h2d_staged_i64).
int h2d_trmv_ops(Engine& E, uint64_t n, const uint8_t* kind, const int64_t* id, const int64_t* score,
                 const uint8_t* dc, const int64_t* ts, uint8_t* kind_d, uint8_t* dc_d, int64_t* id_d,
                 int64_t* score_d, int64_t* ts_d, DevBuf& scratch, DevBuf& dbase) {
  if (!n) return CCRDT_OK;
  static const bool avx2 = __builtin_cpu_supports("avx2");
  const uint64_t n_chunks = (n + OPS_CHUNK - 1) / OPS_CHUNK;
  if (!avx2 || n_chunks > NARROW_MAX_CHUNKS) return CCRDT_ERANGE;
  CCRDT_TRY(stage_init(E));
  CCRDT_TRY(narrow_init(E));
  CCRDT_TRY(scratch.ensure(n * 12));
  CCRDT_TRY(dbase.ensure(n_chunks * 8));
  int64_t* bases = reinterpret_cast<int64_t*>(E.pin_base) + 2 * NARROW_MAX_CHUNKS;
  CCRDT_HIP(hipEventSynchronize(E.pin_bev[2]));
  const int T = (int)std::min<uint64_t>(E.pin_n, n_chunks);
  std::vector<int> rc(T, CCRDT_OK);
  std::vector<std::thread> th;
  th.reserve(T);
  int32_t* d32 = scratch.as<int32_t>();  // [Id | Score | Ts], n each
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      (void)hipSetDevice(E.device);
      char* slot = static_cast<char*>(E.pin[t]);
      int32_t* s32 = reinterpret_cast<int32_t*>(slot);
      uint8_t* s8 = reinterpret_cast<uint8_t*>(slot + OPS_CHUNK * 12);
      for (uint64_t c = (uint64_t)t; c < n_chunks; c += (uint64_t)T) {
        const uint64_t i0 = c * OPS_CHUNK;
        const uint64_t len = std::min<uint64_t>(OPS_CHUNK, n - i0);
        if (hipEventSynchronize(E.pin_ev[t]) != hipSuccess) {
          rc[t] = CCRDT_EDEVICE;
          return;
        }
        int64_t base = 0;
        for (uint64_t i = i0; i < i0 + len; ++i)
          if (kind[i] < 2) {
            base = ts[i];
            break;
          }
        bases[c] = base;
        const bool ok = narrow_stream_avx2(id + i0, nullptr, s32, len, 0) &&
                        narrow_stream_avx2(score + i0, nullptr, s32 + OPS_CHUNK, len, 0) &&
                        narrow_stream_avx2(ts + i0, kind + i0, s32 + 2 * OPS_CHUNK, len, base);
        if (!ok) {
          rc[t] = CCRDT_ERANGE;
          return;
        }
        memcpy(s8, kind + i0, len);
        memcpy(s8 + OPS_CHUNK, dc + i0, len);
        _mm_sfence();
        bool e = false;
        for (int col = 0; col < 3; ++col)
          e = e || hipMemcpyAsync(d32 + col * n + i0, s32 + col * OPS_CHUNK, len * 4, hipMemcpyHostToDevice,
                                  E.stream) != hipSuccess;
        e = e || hipMemcpyAsync(kind_d + i0, s8, len, hipMemcpyHostToDevice, E.stream) != hipSuccess ||
            hipMemcpyAsync(dc_d + i0, s8 + OPS_CHUNK, len, hipMemcpyHostToDevice, E.stream) != hipSuccess ||
            hipEventRecord(E.pin_ev[t], E.stream) != hipSuccess;
        if (e) {
          rc[t] = CCRDT_EDEVICE;
          return;
        }
      }
    });
  for (std::thread& x : th) x.join();
  bool range = false;
  for (int t = 0; t < T; ++t) {
    if (rc[t] == CCRDT_EDEVICE) {
      set_error("h2d_trmv_ops: staging copy failed");
      return rc[t];
    }
    range |= rc[t] == CCRDT_ERANGE;
  }
  if (range) return CCRDT_ERANGE;
  CCRDT_HIP(hipMemcpyAsync(dbase.p, bases, n_chunks * 8, hipMemcpyHostToDevice, E.stream));
  CCRDT_HIP(hipEventRecord(E.pin_bev[2], E.stream));
  return launch_widen_ops(id_d, score_d, ts_d, d32, dbase.as<int64_t>(), kind_d, n, OPS_CHUNK, E.stream);
}

}  // namespace ccrdt
