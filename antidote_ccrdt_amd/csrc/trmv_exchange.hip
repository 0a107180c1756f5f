// trmv_exchange.hip — device side of the two per-batch exchange steps of the
// key-sharded topk_rmv cluster; the collectives themselves are
// RCCL calls of the host (bench.py, cluster.py).
//
//  * replica Vc: the elementwise max of every key's Vc on this shard, the
//    dense-vector form of merge_vcs/2 (src/antidote_ccrdt_topk_rmv.erl:378-386),
//    so that a MAX all-reduce over the shards gives the replica-wide Vc;
//  * extra effects: the {ok, S, [Effect]} effects of the last batch
//    (:236-237, :294-295) packed as int64 rows [op, kind, id, score, dc, ts,
//    vc[0..n_dc)] for the all-gather; rows come out grouped by key (the
//    receiver orders them by op, which is unique).
#include <algorithm>

#include "common.hpp"
#include "trmv_kernels.hpp"

namespace ccrdt {

__global__ __launch_bounds__(256) void trmv_replica_vc_kernel(const int64_t* vc, uint64_t n_keys,
                                                              int n_dc, unsigned long long* out) {
  __shared__ unsigned long long m[TRMV_DPAD];
  if (threadIdx.x < TRMV_DPAD) m[threadIdx.x] = 0ull;
  __syncthreads();
  unsigned long long loc[TRMV_DPAD] = {};
  // Vc entries are >= 0 (0 = absent), so unsigned max is the int64 max
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_keys * (uint64_t)n_dc;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long v = (unsigned long long)vc[i];
    const int d = (int)(i % (uint64_t)n_dc);
#pragma unroll
    for (int k = 0; k < TRMV_DPAD; ++k) loc[k] = (k == d && v > loc[k]) ? v : loc[k];
  }
#pragma unroll
  for (int k = 0; k < TRMV_DPAD; ++k)
    if (k < n_dc && loc[k]) atomicMax(&m[k], loc[k]);
  __syncthreads();
  if ((int)threadIdx.x < n_dc && m[threadIdx.x]) atomicMax(&out[threadIdx.x], m[threadIdx.x]);
}

__global__ __launch_bounds__(256) void trmv_pack_extras_kernel(const uint64_t* key_ptr,
                                                               const uint32_t* ex_cnt,
                                                               const TrmvExtraRec* ex,
                                                               const int64_t* ex_vc, uint64_t n_keys,
                                                               int n_dc, int64_t* rows, int64_t cap,
                                                               uint32_t* count) {
  // (the workgroup's keys reserve their rows with one device atomic: a
  // per-key add on the single count serialized every key with extras)
  __shared__ uint32_t bsum, bbase;
  if (threadIdx.x == 0) bsum = 0u;
  __syncthreads();
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = k < n_keys ? ex_cnt[k] : 0u;
  const uint32_t loc = c ? atomicAdd(&bsum, c) : 0u;
  __syncthreads();
  if (threadIdx.x == 0 && bsum) bbase = atomicAdd(count, bsum);
  __syncthreads();
  if (c == 0) return;
  const uint32_t pos = bbase + loc;
  const uint64_t op0 = key_ptr[k];
  const int w = 6 + n_dc;
  for (uint32_t j = 0; j < c; ++j) {
    const int64_t r = (int64_t)pos + j;
    if (r >= cap) break;
    const TrmvExtraRec e = ex[op0 + j];
    int64_t* row = rows + r * w;
    row[0] = e.op;
    row[1] = e.kind;
    row[2] = e.id;
    row[3] = e.score;
    row[4] = e.dc;
    row[5] = e.ts;
    for (int d = 0; d < n_dc; ++d)
      row[6 + d] = e.kind == CCRDT_TRMV_RMV ? ex_vc[(op0 + j) * n_dc + d] : 0;
  }
}

// The narrow upload's widening (staging.cpp h2d_staged_i64): dst[i] = src[i]
// + (kind == nullptr || kind[i] < 2 ? base[i / chunk] : 0).
__global__ __launch_bounds__(256) void widen_i64_kernel(int64_t* dst, const int32_t* src, const int64_t* base,
                                                        const uint8_t* kind, uint64_t n, uint64_t chunk) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t b = (kind && kind[i] >= 2) ? 0 : base[i / chunk];
    dst[i] = (int64_t)((uint64_t)(int64_t)src[i] + (uint64_t)b);  // (modulo 2^64, as narrowed)
  }
}

int launch_widen_i64(int64_t* dst, const int32_t* src, const int64_t* base, const uint8_t* kind, uint64_t n,
                     uint64_t chunk, hipStream_t st) {
  if (!n) return CCRDT_OK;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(widen_i64_kernel, dim3(blocks), dim3(256), 0, st, dst, src, base, kind, n, chunk);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

// The one-pass upload's widening (staging.cpp h2d_trmv_ops): src = [Id | Score
// | Ts] int32, n each; Ts of adds (kind < 2) plus its chunk's base.
__global__ __launch_bounds__(256) void widen_ops_kernel(int64_t* id, int64_t* score, int64_t* ts, const int32_t* src,
                                                        const int64_t* base, const uint8_t* kind, uint64_t n,
                                                        uint64_t chunk) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    id[i] = (int64_t)src[i];
    score[i] = (int64_t)src[n + i];
    ts[i] = (int64_t)((uint64_t)(int64_t)src[2 * n + i] + (uint64_t)(kind[i] < 2 ? base[i / chunk] : 0));
  }
}

int launch_widen_ops(int64_t* id, int64_t* score, int64_t* ts, const int32_t* src, const int64_t* base,
                     const uint8_t* kind, uint64_t n, uint64_t chunk, hipStream_t st) {
  if (!n) return CCRDT_OK;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(widen_ops_kernel, dim3(blocks), dim3(256), 0, st, id, score, ts, src, base, kind, n, chunk);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_replica_vc(const int64_t* vc, uint64_t n_keys, int n_dc, int64_t* out,
                           hipStream_t st) {
  CCRDT_HIP(hipMemsetAsync(out, 0, (size_t)n_dc * 8, st));
  if (n_keys == 0 || !vc) return CCRDT_OK;
  const uint64_t n = n_keys * (uint64_t)n_dc;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(trmv_replica_vc_kernel, dim3(blocks), dim3(256), 0, st, vc, n_keys, n_dc,
                     (unsigned long long*)out);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

// ------------------------------------------------------ fused exchange
// ------------------------------------------------------ fused exchange
// Extras -> rows with the ops mapped to global ones; the count added into the
// low half of the pack's word 0 (zeroed by the launcher), host_word OR-ed
// into its high half.
__global__ __launch_bounds__(256) void trmv_pack_rows_kernel(const uint64_t* key_ptr, const uint32_t* ex_cnt,
                                                             const TrmvExtraRec* ex, const int64_t* ex_vc,
                                                             uint64_t n_keys, int n_dc, int64_t* pack, int64_t cap,
                                                             const int64_t* op_map, int64_t n_map, uint32_t host_word) {
  __shared__ uint32_t bsum, bbase;
  if (blockIdx.x == 0 && threadIdx.x == 0 && host_word) atomicOr(reinterpret_cast<uint32_t*>(pack) + 1, host_word);
  if (threadIdx.x == 0) bsum = 0u;
  __syncthreads();
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t c = (k < n_keys && ex_cnt) ? ex_cnt[k] : 0u;
  const uint32_t loc = c ? atomicAdd(&bsum, c) : 0u;
  __syncthreads();
  if (threadIdx.x == 0 && bsum) bbase = atomicAdd(reinterpret_cast<uint32_t*>(pack), bsum);  // (low half)
  __syncthreads();
  if (c == 0) return;
  const uint32_t pos = bbase + loc;
  const uint64_t op0 = key_ptr[k];
  const int w = 6 + n_dc;
  int64_t* const rows = pack + 1 + n_dc;
  for (uint32_t j = 0; j < c; ++j) {
    const int64_t r = (int64_t)pos + j;
    if (r >= cap) break;
    const TrmvExtraRec e = ex[op0 + j];
    int64_t* row = rows + r * w;
    row[0] = (op_map && (int64_t)e.op < n_map) ? op_map[e.op] : (int64_t)e.op;
    row[1] = e.kind;
    row[2] = e.id;
    row[3] = e.score;
    row[4] = e.dc;
    row[5] = e.ts;
    for (int d = 0; d < n_dc; ++d) row[6 + d] = e.kind == CCRDT_TRMV_RMV ? ex_vc[(op0 + j) * n_dc + d] : 0;
  }
}

int trmv_launch_replica_vc(const int64_t* vc, uint64_t n_keys, int n_dc, int64_t* out, hipStream_t st);

int trmv_launch_exchange_pack(const int64_t* vc, const uint64_t* key_ptr, const uint32_t* ex_cnt,
                              const TrmvExtraRec* ex, const int64_t* ex_vc, uint64_t n_keys, int n_dc, int64_t* pack,
                              int64_t cap, const int64_t* op_map, int64_t n_map, uint32_t host_word, hipStream_t st) {
  CCRDT_HIP(hipMemsetAsync(pack, 0, 8, st));
  CCRDT_TRY(trmv_launch_replica_vc(vc, n_keys, n_dc, pack + 1, st));
  hipLaunchKernelGGL(trmv_pack_rows_kernel, dim3((unsigned)std::max<uint64_t>((n_keys + 255) / 256, 1)), dim3(256), 0,
                     st, key_ptr, ex_cnt, ex, ex_vc, n_keys, n_dc, pack, cap, op_map, n_map, host_word);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

// The gathered packs -> header + every rank's first rows, sorted by op (a
// stable order: the full 64-bit global op, then the row's (rank, position)
// index, bitonic in one workgroup's LDS; at most 8 ranks x 256 rows per rank
// on this path).
constexpr int XR_MAX = 2048;
__global__ __launch_bounds__(1024) void trmv_exchange_reduce_kernel(const int64_t* g, int world, int64_t len, int n_dc,
                                                                    int64_t* hdr, int64_t* out) {
  __shared__ unsigned long long key[XR_MAX];
  __shared__ uint32_t src[XR_MAX];
  __shared__ uint32_t base[65];
  const int w = 6 + n_dc;
  const int64_t per = (len - 1 - n_dc) / w;
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    uint64_t host = 0;
    for (int r = 0; r < world; ++r) {
      const uint64_t word = (uint64_t)g[r * len];
      const uint32_t c = (uint32_t)(word & 0xFFFFFFFFu);
      hdr[r] = c;
      hdr[world + r] = (int64_t)(word >> 32);
      host += (word >> 32) & 0x3FFFFFFFu;
      base[r] = b;
      b += (uint32_t)(c < per ? c : per);
    }
    base[world] = b;
    hdr[2 * world] = (int64_t)host;
  }
  if (threadIdx.x < (unsigned)n_dc) {
    int64_t m = 0;
    for (int r = 0; r < world; ++r) m = g[r * len + 1 + threadIdx.x] > m ? g[r * len + 1 + threadIdx.x] : m;
    hdr[2 * world + 1 + threadIdx.x] = m;
  }
  __syncthreads();
  const uint32_t n = base[world];
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (uint32_t i = threadIdx.x; i < np2; i += blockDim.x) {
    if (i < n) {
      int r = 0;
      while (base[r + 1] <= i) ++r;
      const uint32_t j = i - base[r];
      const int64_t op = g[r * len + 1 + n_dc + (int64_t)j * w];
      key[i] = (unsigned long long)op;  // i = (rank, position) in rank order: the tie-break
      src[i] = i;
    } else {
      key[i] = ~0ull;
      src[i] = 0xFFFFFFFFu;
    }
  }
  __syncthreads();
  for (uint32_t k = 2; k <= np2; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < np2; i += blockDim.x) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const bool gt = key[i] > key[l] || (key[i] == key[l] && src[i] > src[l]);
          if (gt == up) {
            const unsigned long long t = key[i];
            key[i] = key[l];
            key[l] = t;
            const uint32_t u = src[i];
            src[i] = src[l];
            src[l] = u;
          }
        }
      }
      __syncthreads();
    }
  for (uint32_t i = threadIdx.x; i < n * (uint32_t)w; i += blockDim.x) {
    const uint32_t row = i / w, col = i % w;
    const uint32_t s = src[row];
    int r = 0;
    while (base[r + 1] <= s) ++r;
    out[(int64_t)row * w + col] = g[r * len + 1 + n_dc + (int64_t)(s - base[r]) * w + col];
  }
}

int trmv_launch_exchange_reduce(const int64_t* g, int world, int64_t len, int n_dc, int64_t* hdr, int64_t* out,
                                hipStream_t st) {
  hipLaunchKernelGGL(trmv_exchange_reduce_kernel, dim3(1), dim3(1024), 0, st, g, world, len, n_dc, hdr, out);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

int trmv_launch_pack_extras(const uint64_t* key_ptr, const uint32_t* ex_cnt, const TrmvExtraRec* ex,
                            const int64_t* ex_vc, uint64_t n_keys, int n_dc, int64_t* rows,
                            int64_t cap, uint32_t* count, hipStream_t st) {
  CCRDT_HIP(hipMemsetAsync(count, 0, 4, st));
  if (n_keys == 0 || !ex_cnt) return CCRDT_OK;
  hipLaunchKernelGGL(trmv_pack_extras_kernel, dim3((unsigned)((n_keys + 255) / 256)), dim3(256), 0,
                     st, key_ptr, ex_cnt, ex, ex_vc, n_keys, n_dc, rows, cap, count);
  CCRDT_HIP(hipGetLastError());
  return CCRDT_OK;
}

}  // namespace ccrdt
