// rb_p2p.hip — peer-to-peer position exchange of sharded worlds (SURVEY
// §8e; §7 hard part 4: "a one-shot peer-to-peer all-gather inside a graph").
//
// After the step kernel of step t, every rank's fresh positions sit in its
// own slice of its next snapshot buffer (written back to memory at the step
// kernel's end).  The exchange kernel then
//   1. flags "step t done" to every peer (one system-scope store into the
//      peer's uncached flag array, slot = this rank);
//   2. in every workgroup, waits until every peer has flagged step t (its
//      own uncached flag array, polled by one lane per peer, bounded by a
//      timeout that raises ERR_EXCHANGE instead of hanging; once raised, no
//      later exchange waits);
//   3. reads the other ranks' slices straight from their buffers (IPC
//      mappings over xGMI) into its own buffer and inserts into the next
//      step's table those within a cell of this rank's own bodies' cell
//      bounds (the step kernel folds them, as in halo mode): the only ones
//      an own body can reach next step.
// The buffers alternate with the step parity, and a rank reaches step t+2's
// exchange (which overwrites this parity) only after every peer has flagged
// step t+1, i.e. finished reading it: no further synchronisation is needed.
// Replaces, per step, the all-gather + insert of the RCCL transport.
#include "rb_halo.hpp"

namespace rb {

// a box's orientation row (w x y z) from another GPU's memory
template <typename T> __device__ __forceinline__ void copy_quat_sys(T *dst, const T *src) {
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__global__ __launch_bounds__(256) void p2p_exchange_kernel(P2PParams<T> p) {
    const int64_t e = *p.epoch;
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && tid < p.P && tid != p.rank) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(p.peer_flags[tid] + p.rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (tid < 64) {
        const bool need = tid < p.P && tid != p.rank;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const bool ok = !need || __hip_atomic_load(p.flags + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= e;
            if (__all(ok)) break;
            // bounded: after one timeout (in any exchange) no kernel waits again
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > p.timeout_ticks ||
                (__hip_atomic_load(p.ins.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ERR_EXCHANGE)) {
                if (tid == 0) atomicOr(p.ins.err, ERR_EXCHANGE);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    // the own bodies' cell bounds after this step (the step kernel folded
    // them into BOUND_COPIES copies): a peer body further than a cell from
    // them is out of reach of every own body next step, so it is copied
    // into the snapshot but not inserted (exact: cells are >= 2 x the reach)
    __shared__ int32_t s_b[6];
    if (tid < 64) {
        const int32_t *c = p.bounds + (int64_t)tid * BOUND_STRIDE;
        int32_t b[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) b[d] = c[d];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                b[d] = min(b[d], __shfl_xor(b[d], off));
                b[3 + d] = max(b[3 + d], __shfl_xor(b[3 + d], off));
            }
        if (tid == 0)
#pragma unroll
            for (int d = 0; d < 6; ++d) s_b[d] = b[d];
        if (blockIdx.x == 0) {
            int32_t *r = p.bounds_reset + (int64_t)tid * BOUND_STRIDE;
#pragma unroll
            for (int d = 0; d < 3; ++d) { r[d] = INT32_MAX; r[3 + d] = INT32_MIN; }
        }
    }
    __syncthreads();
    const int64_t id = (int64_t)blockIdx.x * 256 + tid;
    if (id >= p.ins.count || (id >= p.ins.skip_lo && id < p.ins.skip_hi)) return;
    const Snap<T> s = load_snap_sys(p.peer_snap[id / p.S] + id);
    p.dst[id] = s;
    const bool box = p.ins.kind[id] != 0;
    if (box && p.qdst) copy_quat_sys(p.qdst + 4 * id, p.peer_quat[id / p.S] + 4 * id);
    int32_t cx, cy, cz;
    if (!cell_of(s.x, s.y, s.z, p.ins.grid.inv_cs, cx, cy, cz)) return;   // (the owner raised ERR_DOMAIN)
    // empty bounds (min > max: no own body) insert nothing; int64: no overflow at +-1
    if (!(s_b[0] <= s_b[3] && (int64_t)cx >= (int64_t)s_b[0] - 1 && (int64_t)cx <= (int64_t)s_b[3] + 1 &&
          (int64_t)cy >= (int64_t)s_b[1] - 1 && (int64_t)cy <= (int64_t)s_b[4] + 1 &&
          (int64_t)cz >= (int64_t)s_b[2] - 1 && (int64_t)cz <= (int64_t)s_b[5] + 1))
        return;
    insert_id(p.ins.grid, p.ins.tab, p.ins.err, s, (uint32_t)id | (box ? BOX_FLAG : 0u), *p.ins.tab.gen);
}

// ---- halo exchange (large shards) -----------------------------------------
// The step kernel of step e pushes (rb_halo.hpp halo_push): each wave waits
// for the peers' bounds of the step before (published by their insert or
// prime kernels), then appends each own body whose new cell lies within two
// cells of a peer's bounds to that peer's inbox of parity e & 1 (slot from a
// wave-aggregated atomic on push_cnt[peer]), with a box's orientation in box
// worlds, and completes its remote stores before the kernel ends.  Then
//   insert: block 0 reduces the own cell bounds the step kernel folded and
//           stores them, tagged e + 1, into every peer's mailbox (for the
//           peers' next pushes), stores push_cnt[q], tagged e, into peer q's
//           count word of parity e & 1 and resets it, and hands e to the next step kernel
//           (halo_e); every block waits for all peers' counts of step e,
//           then the grid copies the received snapshots (inbox parity e & 1)
//           into the next snapshot buffer and inserts them into the next
//           table;
//   prime:  before a run's first step, the bounds of the current positions,
//           tagged (steps taken) + 1, and halo_e, as an insert kernel of the
//           step before would have left them.
// Publishing the bounds at the start of the insert lets a peer run one step
// ahead: its step e + 1 may push, and its insert e + 1 publish its count,
// while this rank's insert e still reads.  So the inboxes and the count
// words alternate by step parity: a peer writes this rank's parity e & 1
// again only at step e + 2, after this rank's bounds of step e + 1 reached
// it — published by this rank's insert kernel of step e + 1, after its
// insert of step e finished reading.
// Why exact: rb_halo.hpp halo_push.

// One lane per peer (lanes 0..63 of the block) waits until word(q) of every
// peer q != rank carries epoch >= e.  Bounded: after timeout_ticks (or once
// any exchange timed out) ERR_EXCHANGE is raised and the wait ends.
template <typename Word>
__device__ __forceinline__ void wait_peers(int32_t P, int32_t rank, int64_t e, int64_t timeout_ticks, int32_t *err,
                                           Word word) {
    const int tid = threadIdx.x;
    if (tid >= 64) return;
    const bool need = tid < P && tid != rank;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const bool ok = !need || word(tid) >= e;
        if (__all(ok)) break;
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > timeout_ticks ||
            (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ERR_EXCHANGE)) {
            if (tid == 0) atomicOr(err, ERR_EXCHANGE);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// the own cell bounds (lane k folds copy k; the butterfly leaves them in
// every lane), stored tagged into the peers' mailboxes by lanes q < P
template <typename T> __device__ __forceinline__ void publish_bounds(const HaloParams<T> &p, int32_t (&b)[6],
                                                                     int64_t tag) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            b[d] = min(b[d], __shfl_xor(b[d], off));
            b[3 + d] = max(b[3 + d], __shfl_xor(b[3 + d], off));
        }
    if (tid < p.P && tid != p.rank) {
        int64_t *box = reinterpret_cast<int64_t *>(p.peer_mail[tid] + p.lay.o_box) + 6 * p.rank;
#pragma unroll
        for (int d = 0; d < 6; ++d) store_sys(box + d, (int64_t)pack_epoch(tag, b[d]));
    }
}

template <typename T>
__global__ __launch_bounds__(256) void halo_insert_kernel(HaloParams<T> p) {
    const int64_t e = *p.epoch;
    const int tid = threadIdx.x;
    const MailLayout &L = p.lay;
    __shared__ int64_t s_off[65];
    if (blockIdx.x == 0 && tid < 64) {
        const int32_t *c = p.bounds + (int64_t)tid * BOUND_STRIDE;
        int32_t b[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) b[d] = c[d];
        int32_t *r = p.bounds_reset + (int64_t)tid * BOUND_STRIDE;
#pragma unroll
        for (int d = 0; d < 3; ++d) { r[d] = INT32_MAX; r[3 + d] = INT32_MIN; }
        publish_bounds(p, b, e + 1);
        if (tid < p.P && tid != p.rank) {
            // counts by step parity: a peer may reach its next insert (and
            // publish that step's count) while this rank still reads this one
            const int32_t n = p.push_cnt[tid];
            int64_t *cnt = reinterpret_cast<int64_t *>(p.peer_mail[tid] + L.o_cnt) + (e & 1) * p.P + p.rank;
            store_sys(cnt, (int64_t)pack_epoch(e, n < p.S ? n : (int32_t)p.S));
            p.push_cnt[tid] = 0;
        }
        if (tid == 0) *p.halo_e = e;
    }
    const int64_t *cnt_in = reinterpret_cast<const int64_t *>(p.mail + L.o_cnt) + (e & 1) * p.P;
    wait_peers(p.P, p.rank, e, p.timeout_ticks, p.ins.err,
               [&](int q) { return (int64_t)((uint64_t)load_sys(cnt_in + q) >> 32); });
    if (tid == 0) {
        int64_t o = 0;
        for (int q = 0; q < p.P; ++q) {
            s_off[q] = o;
            if (q != p.rank) {
                const int64_t w = load_sys(cnt_in + q);
                // only a current word counts (a timed-out wait leaves stale ones)
                if ((int64_t)((uint64_t)w >> 32) == e) o += (int64_t)(uint32_t)w;
            }
        }
        s_off[p.P] = o;
    }
    __syncthreads();
    const int64_t total = s_off[p.P];
    const int par = (int)(e & 1);
    const uint32_t *ids = reinterpret_cast<const uint32_t *>(p.mail + L.o_ids[par]);
    const Snap<T> *sn = reinterpret_cast<const Snap<T> *>(p.mail + L.o_snap[par]);
    const uint32_t gen = *p.ins.tab.gen;
    for (int64_t k = (int64_t)blockIdx.x * 256 + tid; k < total; k += (int64_t)gridDim.x * 256) {
        int q = 0;
        while (k >= s_off[q + 1]) ++q;
        const int64_t o = (int64_t)q * p.S + (k - s_off[q]);
        const uint32_t id = __hip_atomic_load(ids + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const Snap<T> s = load_snap_sys(sn + o);
        if ((int64_t)id < (int64_t)q * p.S || (int64_t)id >= (int64_t)(q + 1) * p.S) {   // not peer q's body
            atomicOr(p.ins.err, ERR_EXCHANGE);
            continue;
        }
        p.dst[id] = s;
        const bool box = p.ins.kind[id] != 0;
        if (box && p.quat) copy_quat_sys(p.quat + 4 * (int64_t)id, reinterpret_cast<const T *>(p.mail + L.o_quat[par]) + 4 * o);
        insert_id(p.ins.grid, p.ins.tab, p.ins.err, s, id | (box ? BOX_FLAG : 0u), gen);
    }
}

// one block: the own bodies' current cells folded, published tagged
// (steps taken) + 1; halo_e = steps taken
template <typename T>
__global__ __launch_bounds__(256) void halo_prime_kernel(HaloParams<T> p) {
    const int64_t e = *p.epoch;
    const int tid = threadIdx.x;
    int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
    for (int64_t l = tid; l < p.n_local; l += 256) {
        const Snap<T> s = p.own[p.lo + l];
        int32_t c[3];
        if (!cell_of(s.x, s.y, s.z, p.ins.grid.inv_cs, c[0], c[1], c[2])) continue;   // (the step raises ERR_DOMAIN)
#pragma unroll
        for (int d = 0; d < 3; ++d) { lo[d] = min(lo[d], c[d]); hi[d] = max(hi[d], c[d]); }
    }
    __shared__ int32_t s_b[4][6];
    int32_t b[6] = {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            b[d] = min(b[d], __shfl_xor(b[d], off));
            b[3 + d] = max(b[3 + d], __shfl_xor(b[3 + d], off));
        }
    if ((tid & 63) == 0)
#pragma unroll
        for (int d = 0; d < 6; ++d) s_b[tid >> 6][d] = b[d];
    __syncthreads();
    if (tid < 64) {
#pragma unroll
        for (int d = 0; d < 6; ++d) b[d] = s_b[tid & 3][d];   // publish_bounds folds the four waves' results
        publish_bounds(p, b, e + 1);
        if (tid == 0) *p.halo_e = e;
    }
}

template <typename T> hipError_t launch_halo_exchange(const HaloParams<T> &p, hipStream_t s) {
    if (p.P < 1 || p.P > 64 || p.S <= 0) return hipErrorInvalidValue;
    int64_t ib = ((int64_t)(p.P - 1) * p.S + 255) / 256;
    ib = ib < 1 ? 1 : ib > 256 ? 256 : ib;
    hipLaunchKernelGGL((halo_insert_kernel<T>), dim3((unsigned)ib), dim3(256), 0, s, p);
    return hipGetLastError();
}
template <typename T> hipError_t launch_halo_prime(const HaloParams<T> &p, hipStream_t s) {
    if (p.P < 1 || p.P > 64 || p.S <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL((halo_prime_kernel<T>), dim3(1), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename T> hipError_t launch_p2p_exchange(const P2PParams<T> &p, hipStream_t s) {
    if (p.ins.count <= 0 || p.P < 1 || p.P > 64) return hipErrorInvalidValue;
    const int64_t blocks = (p.ins.count + 255) / 256;
    hipLaunchKernelGGL((p2p_exchange_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t launch_p2p_exchange<double>(const P2PParams<double> &, hipStream_t);
template hipError_t launch_p2p_exchange<float>(const P2PParams<float> &, hipStream_t);
template hipError_t launch_halo_exchange<double>(const HaloParams<double> &, hipStream_t);
template hipError_t launch_halo_exchange<float>(const HaloParams<float> &, hipStream_t);
template hipError_t launch_halo_prime<double>(const HaloParams<double> &, hipStream_t);
template hipError_t launch_halo_prime<float>(const HaloParams<float> &, hipStream_t);

}  // namespace rb

// ---- the error word to the host (rb_sync, rb_step) ----------------------------
// One lane stores the device error word into pinned, device-mapped host memory
// (a system-scope vector store), so the host reads it after the stream
// synchronises without a device-to-host copy behind the stream's work; tile
// runs' graphs also publish the tile form's reason bits and commit count.
namespace rb {
__global__ __launch_bounds__(64) void publish_err_kernel(const int32_t *err, int32_t *host, const int32_t *why,
                                                         const unsigned long long *commits, int64_t *host_tile) {
    if (threadIdx.x == 0) {
        __hip_atomic_store(host, __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        if (why) {
            const int64_t wv = __hip_atomic_load(why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int64_t cv = (int64_t)__hip_atomic_load(commits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(host_tile, wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_tile + 1, cv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
hipError_t launch_publish_err(const int32_t *err, int32_t *host_dev, hipStream_t s, const int32_t *why,
                              const unsigned long long *commits, int64_t *host_tile_dev) {
    hipLaunchKernelGGL(publish_err_kernel, dim3(1), dim3(64), 0, s, err, host_dev, why, commits, host_tile_dev);
    return hipGetLastError();
}
}  // namespace rb
