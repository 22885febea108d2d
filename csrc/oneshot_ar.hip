// K9: one-shot all-reduce for tensor-parallel decode over xGMI.
//
// A decode all-reduce is tiny ([B, hidden] bf16: 16 KB at B = 1 on Llama-3-70B) and there are
// two per layer (160 per token at TP = 4). RCCL's ring spends world-1 dependent steps per call;
// on MI355X every GPU has a dedicated xGMI link to each peer, so one step suffices: every rank
// PUSHES its slice straight into every peer's receive buffer (posted remote writes, one link per
// peer, all links at once), raises one flag per (peer, workgroup), waits for the peers' flags in
// its own memory, and sums the world copies locally in rank order (bit-identical results on
// every rank, like RCCL).
//
// Memory: receive buffers and flags are hipDeviceMallocUncached (fine-grained, never cached in a
// GPU's L2/MALL, so a remote write is what the next local load sees) and exported to the peers
// with hipIpcGetMemHandle (dmabuf) / hipIpcOpenMemHandle. Two slots alternate by call parity:
// before rank r writes slot s again (call e), it has seen every peer's flag of call e-1, which
// each peer raised only after its call e-2 — the last reader of slot s — had finished.
// The call counter (`epoch`) lives on the device and is advanced by the last workgroup out, so
// the launch is hipGraph-capturable and replays with no host involvement.
// Every flag wait is bounded: on expiry *err is set and the kernel proceeds (never a hang).
//
// LL form (oneshot_ar_ll_kernel, chosen per node by a timed probe, parallel/oneshot.py): every
// 4-byte word of the slice travels with the call's epoch in ONE 8-byte store ((data, epoch)
// pairs), so a receiver polls the data itself. The flag form pays, after its pushes, a system
// fence (every remote store acknowledged: an xGMI round trip), then the flag's one-way trip,
// then a local read of the data; the LL form pays the data's one-way trip only, for twice the
// bytes on the link (a decode all-reduce is 24 KB: ~0.5 us more at ~50 GB/s per link).
//
// The same comm also serves the FUSED form (skinny_gemm_ar_kernel below, epilogue EPI_AR of
// skinny_core.h): a row-parallel decode GEMM (o / down projection) exchanges each finished
// 16-column tile itself — push, per-(peer, tile) flag, wait, rank-order sum — so the decode step
// has no separate all-reduce launch at all, and a tile's xGMI round trip overlaps the other
// tiles' weight streams. Both forms share the receive buffers and the call counter (a call of
// either kind is one epoch), so they interleave freely within a captured graph.
#include "skinny_core.h"

#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

namespace {
constexpr int MAXW = 8;    // ranks per all-reduce group (one xGMI hop to every peer)
constexpr int MAXB = 64;   // workgroups per call (flags per (slot, source rank))
constexpr long long FLAG_POLL_LIMIT = 1ll << 26;   // default bound (~seconds); tests lower it per comm
constexpr int MAXT = 1024; // 16-column tiles per fused call (N <= 16384)
constexpr int GCAP = 16 * 131072;   // all-gather output elements per slot (16 rows x a 128K vocab)
constexpr int NHANDLES = 6;         // IPC handles per rank: data, flags, tile flags, gather data, gather flags, LL
static_assert(MAXW == skinny::AR_MAXW, "rank limit shared with the fused epilogue");

struct Peers {
  uint16_t* data[MAXW];    // rank p's receive buffer: [2 slots][world][cap] bf16
  uint32_t* flags[MAXW];   // rank p's flags: [2 slots][world][MAXB]
};

// res != nullptr: the residual form — the sum is rounded to bf16 and added into res in place,
// res = bf16(res + bf16(sum)) (exactly what the next layer's NORM_ADD prologue used to form), and
// `inout` is left as it was; the next GEMM then reads res with a plain NORM prologue.
__global__ void __launch_bounds__(256) oneshot_ar_kernel(uint16_t* __restrict__ inout, int n, int rank, int world,
                                                         int cap, Peers P, uint32_t* epoch_ctr, uint32_t* done_ctr,
                                                         int* err, long long poll_limit, uint16_t* __restrict__ res) {
  const uint32_t epoch = __hip_atomic_load(epoch_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int slot = (int)(epoch & 1u);
  const int nb = gridDim.x, blk = blockIdx.x;
  const int nvec = n >> 3;                              // 16-byte vectors
  const int per = (nvec + nb - 1) / nb;
  const int v0 = blk * per, v1 = min(nvec, v0 + per);
  using rt::float4_;
  using vec = uint4;

  // 1. push this workgroup's slice into every rank's receive buffer (own rank included)
  for (int v = v0 + (int)threadIdx.x; v < v1; v += blockDim.x) {
    const vec x = reinterpret_cast<const vec*>(inout)[v];
    for (int p = 0; p < world; ++p)
      reinterpret_cast<vec*>(P.data[p] + ((size_t)slot * world + rank) * cap)[v] = x;
  }
  // 2. release: every thread's remote stores complete before any flag is raised
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world)
    __hip_atomic_store(P.flags[threadIdx.x] + ((size_t)slot * world + rank) * MAXB + blk, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every rank's copy of this slice in our own memory
  if ((int)threadIdx.x < world) {
    const uint32_t* f = P.flags[rank] + ((size_t)slot * world + threadIdx.x) * MAXB + blk;
    long long it = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > poll_limit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  // 4. sum the world copies in rank order (fp32), write the result in place
  const uint16_t* mine = P.data[rank] + (size_t)slot * world * cap;
  for (int v = v0 + (int)threadIdx.x; v < v1; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < world; ++r) {
      const vec x = reinterpret_cast<const vec*>(mine + (size_t)r * cap)[v];
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += rt::bf2f((uint16_t)(w[j] & 0xffffu));
        acc[2 * j + 1] += rt::bf2f((uint16_t)(w[j] >> 16));
      }
    }
    if (res != nullptr) {
      const vec rv = reinterpret_cast<const vec*>(res)[v];
      const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] = rt::bf2f((uint16_t)(rw[j] & 0xffffu)) + rt::bf2f(rt::f2bf(acc[2 * j]));
        acc[2 * j + 1] = rt::bf2f((uint16_t)(rw[j] >> 16)) + rt::bf2f(rt::f2bf(acc[2 * j + 1]));
      }
    }
    vec o;
    o.x = rt::pack2(acc[0], acc[1]);
    o.y = rt::pack2(acc[2], acc[3]);
    o.z = rt::pack2(acc[4], acc[5]);
    o.w = rt::pack2(acc[6], acc[7]);
    reinterpret_cast<vec*>(res != nullptr ? res : inout)[v] = o;
  }
  // 5. the last workgroup out advances the call counter (every workgroup has read it)
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)nb - 1u) {
      __hip_atomic_store(done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(epoch_ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct LLPeers {
  uint64_t* ll[MAXW];      // rank p's LL buffer: [2 slots][world][cap / 2] (data word, epoch) pairs
};

__global__ void __launch_bounds__(256) oneshot_ar_ll_kernel(uint16_t* __restrict__ inout, int n, int rank, int world,
                                                            int cap, LLPeers P, uint32_t* epoch_ctr,
                                                            uint32_t* done_ctr, int* err, long long poll_limit,
                                                            uint16_t* __restrict__ res) {
  const uint32_t epoch = __hip_atomic_load(epoch_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int slot = (int)(epoch & 1u);
  const int nb = gridDim.x, blk = blockIdx.x;
  const int nvec = n >> 3;                              // 16-byte vectors (4 pairs each)
  const int per = (nvec + nb - 1) / nb;
  const int v0 = blk * per, v1 = min(nvec, v0 + per);
  const size_t rstride = (size_t)cap / 2;               // pairs per (slot, source rank)
  const uint64_t tag = (uint64_t)epoch << 32;
  // 1. push: four 8-byte (word, epoch) stores per vector into every rank's buffer (own included)
  for (int v = v0 + (int)threadIdx.x; v < v1; v += blockDim.x) {
    const uint4 x = reinterpret_cast<const uint4*>(inout)[v];
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
    for (int p = 0; p < world; ++p) {
      uint64_t* dst = P.ll[p] + ((size_t)slot * world + rank) * rstride + 4 * (size_t)v;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __hip_atomic_store(dst + j, tag | w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // 2. receive: every rank's 4 pairs of the vector requested at once, re-polled until each
  // carries this call's epoch (bounded), then summed in rank order (bit-identical on every rank)
  const uint64_t* mine = P.ll[rank] + (size_t)slot * world * rstride;
  for (int v = v0 + (int)threadIdx.x; v < v1; v += blockDim.x) {
    uint64_t q[MAXW][4];
#pragma unroll
    for (int r = 0; r < MAXW; ++r)
      if (r < world)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          q[r][j] = __hip_atomic_load(mine + (size_t)r * rstride + 4 * (size_t)v + j, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
    for (int r = 0; r < MAXW; ++r) {
      if (r >= world) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        long long it = 0;
        while ((uint32_t)(q[r][j] >> 32) != epoch) {
          __builtin_amdgcn_s_sleep(1);
          if (++it > poll_limit) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          q[r][j] = __hip_atomic_load(mine + (size_t)r * rstride + 4 * (size_t)v + j, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < MAXW; ++r) {
      if (r >= world) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wj = (uint32_t)q[r][j];
        acc[2 * j] += rt::bf2f((uint16_t)(wj & 0xffffu));
        acc[2 * j + 1] += rt::bf2f((uint16_t)(wj >> 16));
      }
    }
    if (res != nullptr) {
      const uint4 rv = reinterpret_cast<const uint4*>(res)[v];
      const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] = rt::bf2f((uint16_t)(rw[j] & 0xffffu)) + rt::bf2f(rt::f2bf(acc[2 * j]));
        acc[2 * j + 1] = rt::bf2f((uint16_t)(rw[j] >> 16)) + rt::bf2f(rt::f2bf(acc[2 * j + 1]));
      }
    }
    uint4 o;
    o.x = rt::pack2(acc[0], acc[1]);
    o.y = rt::pack2(acc[2], acc[3]);
    o.z = rt::pack2(acc[4], acc[5]);
    o.w = rt::pack2(acc[6], acc[7]);
    reinterpret_cast<uint4*>(res != nullptr ? res : inout)[v] = o;
  }
  // 3. the last workgroup out advances the call counter (every workgroup has read it)
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)nb - 1u) {
      __hip_atomic_store(done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(epoch_ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One-shot ALL-GATHER (C3: the vocab-parallel logits of a tensor-parallel decode step): every
// rank pushes its [rows, shard] slice straight into its column block of every rank's
// [rows, world * shard] receive buffer, raises one flag per (peer, workgroup), waits for the
// peers' flags of the same workgroup range and copies the gathered rows out — one launch and
// one xGMI hop, replacing RCCL's ring all-gather plus the permute into [rows, world * shard].
// Same epoch / slot discipline as the all-reduce (shared call counter).
struct GPeers {
  uint16_t* data[MAXW];    // rank p's gather buffer: [2 slots][GCAP]
  uint32_t* flags[MAXW];   // rank p's gather flags: [2 slots][world][MAXB]
};

__global__ void __launch_bounds__(256) oneshot_ag_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                         int rows, int shard, int rank, int world, GPeers P,
                                                         uint32_t* epoch_ctr, uint32_t* done_ctr, int* err,
                                                         long long poll_limit) {
  const uint32_t epoch = __hip_atomic_load(epoch_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int slot = (int)(epoch & 1u);
  const int nb = gridDim.x, blk = blockIdx.x;
  const int vrow = shard >> 3;                          // 16-byte vectors per row of a slice
  const int nvec = rows * vrow;
  const int per = (nvec + nb - 1) / nb;
  const int v0 = blk * per, v1 = min(nvec, v0 + per);
  const size_t ld = (size_t)world * shard;              // gathered row length
  using vec = uint4;
  // 1. push this workgroup's vectors of our slice into every rank's buffer (own included)
  for (int v = v0 + (int)threadIdx.x; v < v1; v += blockDim.x) {
    const int row = v / vrow, c8 = v - row * vrow;
    const vec x = reinterpret_cast<const vec*>(in)[v];
    const size_t dst = (size_t)slot * GCAP + row * ld + (size_t)rank * shard + (size_t)c8 * 8;
    for (int p = 0; p < world; ++p) *reinterpret_cast<vec*>(P.data[p] + dst) = x;
  }
  __threadfence_system();
  __syncthreads();
  if ((int)threadIdx.x < world)
    __hip_atomic_store(P.flags[threadIdx.x] + ((size_t)slot * world + rank) * MAXB + blk, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 2. wait for every rank's vectors of the same range (every rank's slice has the same shape)
  if ((int)threadIdx.x < world) {
    const uint32_t* f = P.flags[rank] + ((size_t)slot * world + threadIdx.x) * MAXB + blk;
    long long it = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > poll_limit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __syncthreads();
  // 3. copy the gathered range of every rank's block out of the (uncached) receive buffer
  const uint16_t* mine = P.data[rank] + (size_t)slot * GCAP;
  for (int r = 0; r < world; ++r)
    for (int v = v0 + (int)threadIdx.x; v < v1; v += blockDim.x) {
      const int row = v / vrow, c8 = v - row * vrow;
      const size_t o = row * ld + (size_t)r * shard + (size_t)c8 * 8;
      reinterpret_cast<vec*>(out + o)[0] = *reinterpret_cast<const vec*>(mine + o);
    }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)nb - 1u) {
      __hip_atomic_store(done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(epoch_ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct Comm {
  int world = 0, rank = 0, cap = 0;       // cap: max elements per call
  int device = 0;
  uint16_t* data = nullptr;               // own receive buffer
  uint32_t* flags = nullptr;              // own flags
  uint32_t* tflags = nullptr;             // own per-tile flags of the fused GEMM form
  uint32_t* peer_tflags[MAXW] = {};
  uint16_t* gdata = nullptr;              // own all-gather buffer
  uint32_t* gflags = nullptr;             // own all-gather flags
  GPeers gpeers{};
  uint32_t* ctr = nullptr;                // [epoch, done] (plain device memory, local only)
  int* err = nullptr;
  long long poll_limit = FLAG_POLL_LIMIT;
  uint64_t* ll = nullptr;                 // own LL receive buffer
  LLPeers llpeers{};
  int use_ll = 0;                         // the all-reduce launch takes the LL form
  Peers peers{};
  std::vector<void*> opened;              // IPC mappings to close
};
std::mutex g_mu;
std::vector<Comm*> g_comms;

Comm* get(int id) {
  std::lock_guard<std::mutex> lk(g_mu);
  return (id >= 0 && id < (int)g_comms.size()) ? g_comms[id] : nullptr;
}
size_t data_bytes(const Comm& c) { return (size_t)2 * c.world * c.cap * sizeof(uint16_t); }
size_t flag_bytes(const Comm& c) { return (size_t)2 * c.world * MAXB * sizeof(uint32_t); }
size_t tflag_bytes(const Comm& c) { return (size_t)2 * c.world * MAXT * sizeof(uint32_t); }
size_t gdata_bytes() { return (size_t)2 * GCAP * sizeof(uint16_t); }
size_t ll_bytes(const Comm& c) { return (size_t)2 * c.world * (c.cap / 2) * sizeof(uint64_t); }

template <int NW, int U>
__global__ void __launch_bounds__(NW * 64) skinny_gemm_ar_kernel(skinny::GemmArgs p) {
  __shared__ skinny::GemmSmem<1, NW> sm;
  skinny::Stage<skinny::PRO_PLAIN, skinny::EPI_AR, U> st0;
  skinny::gemm_tile<skinny::PRO_PLAIN, skinny::EPI_AR, NW, U, false>(p, blockIdx.x, sm, st0, false, false);
}
}  // namespace

// Allocates this rank's IPC buffers. Returns a comm id (>= 0) or a negative error; the
// NHANDLES 64-byte IPC handles (data, flags, tile flags, gather data, gather flags, LL) are written
// to `handles` (64 * NHANDLES bytes).
int oneshot_create(int world, int rank, int cap_elems, char* handles) {
  if (world < 2 || world > MAXW || rank < 0 || rank >= world || cap_elems < 8 || cap_elems % 8) return -1;
  Comm* c = new Comm;
  c->world = world;
  c->rank = rank;
  c->cap = cap_elems;
  if (hipGetDevice(&c->device) != hipSuccess) { delete c; return -2; }
  if (hipExtMallocWithFlags((void**)&c->data, data_bytes(*c), hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&c->flags, flag_bytes(*c), hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&c->tflags, tflag_bytes(*c), hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&c->gdata, gdata_bytes(), hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&c->gflags, flag_bytes(*c), hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void**)&c->ll, ll_bytes(*c), hipDeviceMallocUncached) != hipSuccess ||
      hipMalloc((void**)&c->ctr, 2 * sizeof(uint32_t)) != hipSuccess || hipMalloc((void**)&c->err, sizeof(int)) != hipSuccess) {
    delete c;
    return -3;
  }
  if (hipMemset(c->flags, 0, flag_bytes(*c)) != hipSuccess || hipMemset(c->tflags, 0, tflag_bytes(*c)) != hipSuccess ||
      hipMemset(c->gflags, 0, flag_bytes(*c)) != hipSuccess || hipMemset(c->ll, 0, ll_bytes(*c)) != hipSuccess ||
      hipMemset(c->ctr, 0, 2 * sizeof(uint32_t)) != hipSuccess ||
      hipMemset(c->err, 0, sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    delete c;
    return -4;
  }
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  void* const bufs[NHANDLES] = {c->data, c->flags, c->tflags, c->gdata, c->gflags, c->ll};
  for (int i = 0; i < NHANDLES; ++i) {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, bufs[i]) != hipSuccess) {
      delete c;
      return -5;
    }
    memcpy(handles + 64 * i, &h, 64);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  return (int)g_comms.size() - 1;
}

// Maps every peer's buffers: `all_handles` = world x (64 * NHANDLES) bytes, in rank order.
int oneshot_open(int id, const char* all_handles) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  for (int p = 0; p < c->world; ++p) {
    void* b[NHANDLES] = {c->data, c->flags, c->tflags, c->gdata, c->gflags, c->ll};
    if (p != c->rank) {
      for (int i = 0; i < NHANDLES; ++i) {
        hipIpcMemHandle_t h;
        memcpy(&h, all_handles + (size_t)p * 64 * NHANDLES + 64 * i, 64);
        if (hipIpcOpenMemHandle(&b[i], h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -2 - i;
        c->opened.push_back(b[i]);
      }
    }
    c->peers.data[p] = (uint16_t*)b[0];
    c->peers.flags[p] = (uint32_t*)b[1];
    c->peer_tflags[p] = (uint32_t*)b[2];
    c->gpeers.data[p] = (uint16_t*)b[3];
    c->gpeers.flags[p] = (uint32_t*)b[4];
    c->llpeers.ll[p] = (uint64_t*)b[5];
  }
  return 0;
}

int oneshot_handle_bytes() { return 64 * NHANDLES; }

int oneshot_capacity(int id) {
  Comm* c = get(id);
  return c ? c->cap : -1;
}

// In-place sum over the group of `n` bf16 elements at `inout` (device pointer, 16-B aligned).
// res (optional, [n] bf16, 16-B aligned): the residual form (see oneshot_ar_kernel).
int oneshot_allreduce(int id, void* inout, int n, void* res, hipStream_t stream) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  if (n <= 0 || n % 8 || n > c->cap || ((uintptr_t)inout & 15) || ((uintptr_t)res & 15)) return -2;
  for (int p = 0; p < c->world; ++p)
    if (c->peers.data[p] == nullptr) return -3;   // oneshot_open not called
  int nb = n / 2048;                                // ~4 KB of slice per workgroup
  nb = nb < 1 ? 1 : (nb > MAXB ? MAXB : nb);
  if (c->use_ll) {
    if (c->llpeers.ll[c->rank] == nullptr) return -3;
    hipLaunchKernelGGL(oneshot_ar_ll_kernel, dim3(nb), dim3(256), 0, stream, (uint16_t*)inout, n, c->rank, c->world,
                       c->cap, c->llpeers, c->ctr, c->ctr + 1, c->err, c->poll_limit, (uint16_t*)res);
  } else {
    hipLaunchKernelGGL(oneshot_ar_kernel, dim3(nb), dim3(256), 0, stream, (uint16_t*)inout, n, c->rank, c->world,
                       c->cap, c->peers, c->ctr, c->ctr + 1, c->err, c->poll_limit, (uint16_t*)res);
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Fused row-parallel decode GEMM + all-reduce: out[M, N] = sum over ranks of x_r[M, K] . W_r[N, K]^T,
// every rank calling with its own shard (Ws shuffled by shuffle_weight, plain layout rule).
// Same (NW, U) rule as the standalone plain launch (gemm_skinny.hip): 4 x 4 below 384 tiles.
// res (optional, [M, N] bf16): the residual form — res = bf16(res + bf16(sum)) in place, `out`
// untouched (may be null).
int oneshot_gemm_ar(int id, void* out, const void* x, const void* Ws, int M, int N, int K, void* res,
                    hipStream_t stream) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  if (M < 1 || M > 16 || K % 32 || N % 16 || N / 16 > MAXT || (int64_t)M * N > c->cap) return -2;
  if (((uintptr_t)out & 15) || ((uintptr_t)x & 15) || ((uintptr_t)Ws & 15)) return -2;
  if (out == nullptr && res == nullptr) return -2;
  for (int p = 0; p < c->world; ++p)
    if (c->peers.data[p] == nullptr || c->peer_tflags[p] == nullptr) return -3;
  skinny::GemmArgs args{(uint16_t*)out, (const uint16_t*)x, (const rt::short8*)Ws, (uint16_t*)res, M, N, K, N, 0.f,
                        skinny::RopeEpi{}, nullptr, nullptr};
  for (int p = 0; p < c->world; ++p) {
    args.ar.data[p] = c->peers.data[p];
    args.ar.tflags[p] = c->peer_tflags[p];
    args.ar.ll[p] = c->llpeers.ll[p];
  }
  args.ar.use_ll = c->use_ll;
  args.ar.ctr = c->ctr;
  args.ar.err = c->err;
  args.ar.poll_limit = c->poll_limit;
  args.ar.rank = c->rank;
  args.ar.world = c->world;
  args.ar.cap = c->cap;
  args.ar.maxt = MAXT;
  const dim3 grid(N / 16);
  if (N / 16 >= 384)
    hipLaunchKernelGGL((skinny_gemm_ar_kernel<4, 2>), grid, dim3(256), 0, stream, args);
  else
    hipLaunchKernelGGL((skinny_gemm_ar_kernel<4, 4>), grid, dim3(256), 0, stream, args);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// All-gather along the last dim: out[rows, world * shard] <- every rank's in[rows, shard].
int oneshot_allgather(int id, const void* in, void* out, int rows, int shard, hipStream_t stream) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  if (rows < 1 || shard < 8 || shard % 8 || (int64_t)rows * shard * c->world > GCAP) return -2;
  if (((uintptr_t)in & 15) || ((uintptr_t)out & 15)) return -2;
  for (int p = 0; p < c->world; ++p)
    if (c->gpeers.data[p] == nullptr) return -3;
  const int nvec = rows * (shard / 8);
  int nb = (nvec + 255) / 256;                      // one 16-B vector per thread per peer
  nb = nb < 1 ? 1 : (nb > MAXB ? MAXB : nb);
  hipLaunchKernelGGL(oneshot_ag_kernel, dim3(nb), dim3(256), 0, stream, (const uint16_t*)in, (uint16_t*)out, rows,
                     shard, c->rank, c->world, c->gpeers, c->ctr, c->ctr + 1, c->err, c->poll_limit);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

int oneshot_gather_capacity() { return GCAP; }

// Poll-expiry flag (1 = a peer's flag never arrived: results of that call are wrong).
int oneshot_error(int id) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  int e = 0;
  if (hipMemcpy(&e, c->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  return e;
}

// Clears the poll-expiry flag after the host has failed the affected turn.
int oneshot_clear_error(int id) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  return hipMemset(c->err, 0, sizeof(int)) == hipSuccess && hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}

// This rank's device call counter (the epoch of its last completed call). Host read, synchronous.
long long oneshot_epoch(int id) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  uint32_t e = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&e, c->ctr, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return -2;
  return (long long)e;
}

// Re-arm this rank's side of the comm at an epoch the group agreed on (parallel/oneshot.py
// resync: every rank quiesced and past a group barrier, then this, then a second barrier): the call
// counter becomes `epoch`, the done counter and the expiry flag 0, and every receive buffer this
// rank owns — flags, tile flags, gather flags, LL (word, epoch) pairs — is zeroed, so no stale tag
// of a call some rank issued alone can match a future epoch. Local memory only.
int oneshot_resync(int id, long long epoch) {
  Comm* c = get(id);
  if (c == nullptr || epoch < 0 || epoch > 0xffffffffll) return -1;
  const uint32_t ctr[2] = {(uint32_t)epoch, 0u};
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemset(c->flags, 0, flag_bytes(*c)) != hipSuccess || hipMemset(c->tflags, 0, tflag_bytes(*c)) != hipSuccess ||
      hipMemset(c->gflags, 0, flag_bytes(*c)) != hipSuccess || hipMemset(c->ll, 0, ll_bytes(*c)) != hipSuccess ||
      hipMemcpy(c->ctr, ctr, sizeof(ctr), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->err, 0, sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return -3;
  return 0;
}

// ---- device-side stand-in for a collective (bench.py --simulate-tp, parallel/tp.py SimulatedTP) ----
// One process computes rank 0's shard of a tp = N engine; every collective becomes this kernel: `nb`
// workgroups (the K9 launch's own count for the message) each hold their CU for `ticks` of the
// 100 MHz s_memrealtime clock, then exit — the step pays the collective's latency INSIDE the captured
// graph, on the stream, occupying the CUs a real K9 call occupies, so a schedule that overlaps
// communication with other work (a second stream) can be measured on one GPU.
__global__ void __launch_bounds__(64) sim_comm_spin_kernel(long long ticks) {
  if (threadIdx.x != 0) return;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

int sim_comm_spin(long long ticks, int nb, hipStream_t stream) {
  if (nb < 1 || nb > 1024 || ticks < 0) return -1;
  hipLaunchKernelGGL(sim_comm_spin_kernel, dim3(nb), dim3(64), 0, stream, ticks);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Flag-wait bound in poll iterations (fault-injection tests force an expiry with a tiny bound).
int oneshot_set_poll_limit(int id, long long limit) {
  Comm* c = get(id);
  if (c == nullptr || limit < 1) return -1;
  c->poll_limit = limit;
  return 0;
}

// Protocol of the all-reduce launch and of the fused GEMM form: 1 = LL (data + epoch pairs),
// 0 = push + fence + flag. (The all-gather keeps the flag form: its payload is 4x larger.)
int oneshot_set_ll(int id, int on) {
  Comm* c = get(id);
  if (c == nullptr) return -1;
  c->use_ll = on ? 1 : 0;
  return 0;
}

void oneshot_destroy(int id) {
  Comm* c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (id < 0 || id >= (int)g_comms.size()) return;
    c = g_comms[id];
    g_comms[id] = nullptr;
  }
  if (c == nullptr) return;
  (void)hipDeviceSynchronize();
  for (void* p : c->opened) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(c->data);
  (void)hipFree(c->flags);
  (void)hipFree(c->tflags);
  (void)hipFree(c->gdata);
  (void)hipFree(c->gflags);
  (void)hipFree(c->ll);
  (void)hipFree(c->ctr);
  (void)hipFree(c->err);
  delete c;
}
