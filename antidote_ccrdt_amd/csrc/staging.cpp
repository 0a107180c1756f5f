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
#include <cstring>
#include <thread>
#include <vector>

#include "engine.hpp"

namespace ccrdt {

namespace {
constexpr int STAGE_THREADS = 8;
constexpr uint64_t STAGE_CHUNK = 16ull << 20;          // bytes per slot
constexpr uint64_t STAGE_DIRECT = 4ull << 20;           // below: one plain copy
}  // namespace

static int stage_init(Engine& E) {
  if (E.pin_n) return CCRDT_OK;
  for (int t = 0; t < STAGE_THREADS; ++t) {
    CCRDT_HIP(hipHostMalloc(&E.pin[t], STAGE_CHUNK, hipHostMallocDefault));
    CCRDT_HIP(hipEventCreateWithFlags(&E.pin_ev[t], hipEventDisableTiming));
    CCRDT_HIP(hipEventRecord(E.pin_ev[t], E.stream));  // "slot free"
    E.pin_n = t + 1;
  }
  return CCRDT_OK;
}

void stage_release(Engine& E) {
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
  const int T = (int)std::min<uint64_t>(STAGE_THREADS, n_chunks);
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
