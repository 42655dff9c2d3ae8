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
//      mappings over xGMI) into its own buffer and inserts those bodies into
//      the next step's table.
// The buffers alternate with the step parity, and a rank reaches step t+2's
// exchange (which overwrites this parity) only after every peer has flagged
// step t+1, i.e. finished reading it: no further synchronisation is needed.
// Replaces, per step, the all-gather + insert of the RCCL transport.
#include "rb_grid.hpp"

namespace rb {

// System-scope word accesses: they bypass the caches on both sides, so data
// another GPU wrote (or will read) needs no cache maintenance — no L2
// writeback or invalidate (a fence per wave or block at agent/system scope
// costs an L2 writeback/invalidate each: measured +9-13 us per step at C3).
__device__ __forceinline__ int64_t load_sys(const int64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void store_sys(int64_t *p, int64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T> __device__ __forceinline__ Snap<T> load_snap_sys(const Snap<T> *p) {
    const T *w = &p->x;
    Snap<T> s;
    s.x = __hip_atomic_load(w + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s.y = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s.z = __hip_atomic_load(w + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s.r = __hip_atomic_load(w + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return s;
}
template <typename T> __device__ __forceinline__ void store_snap_sys(Snap<T> *p, const Snap<T> &s) {
    T *w = &p->x;
    __hip_atomic_store(w + 0, s.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(w + 1, s.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(w + 2, s.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(w + 3, s.r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

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
    __syncthreads();
    const int64_t id = (int64_t)blockIdx.x * 256 + tid;
    if (id >= p.ins.count || (id >= p.ins.skip_lo && id < p.ins.skip_hi)) return;
    const Snap<T> s = load_snap_sys(p.peer_snap[id / p.S] + id);
    p.dst[id] = s;
    const bool box = p.ins.kind[id] != 0;
    if (box && p.qdst) copy_quat_sys(p.qdst + 4 * id, p.peer_quat[id / p.S] + 4 * id);
    insert_id(p.ins.grid, p.ins.tab, p.ins.err, s, (uint32_t)id | (box ? BOX_FLAG : 0u), *p.ins.tab.gen);
}

// ---- halo exchange (large shards) -----------------------------------------
// Two kernels after the step kernel of step e (HaloParams, rb_internal.hpp):
//   push:   block 0 reduces the own cell bounds and stores them, epoch-tagged,
//           into every peer's mailbox (and resets the other parity's copies);
//           every block waits for all peers' bounds of step e, then each
//           thread tests one own body's new cell against each peer's bounds
//           +-1 cell and, if inside, appends (id, snapshot) to that peer's
//           inbox (slot from a wave-aggregated atomic on push_cnt[peer]),
//           with a box's orientation in box worlds;
//           each wave ends with a system-scope release (its remote stores
//           complete before the kernel does);
//   insert: block 0 stores push_cnt[q], epoch-tagged, into peer q's mailbox
//           and resets it; every block waits for all peers' counts of step
//           e, then the grid copies the received snapshots into the next
//           snapshot buffer and inserts them into the next table.
// A peer pushes into this rank's inbox for step e+1 only after this rank's
// bounds of step e+1 reached it, i.e. after this rank's insert of step e
// finished reading: one inbox per peer suffices.
// Why exact: a partner j of an own body i lies within reach of i, and the
// cell size is >= 2 x the reach, so cell(j) is within one cell of cell(i)
// on every axis — inside the bounds +-1 of i's rank.  Bodies not pushed are
// never within reach of any body of the receiving rank, and every contact
// test and its order depend only on the bodies within reach.

__device__ __forceinline__ uint64_t pack_epoch(int64_t e, int32_t v) {
    return ((uint64_t)e << 32) | (uint32_t)v;
}

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


template <typename T>
__global__ __launch_bounds__(256) void halo_push_kernel(HaloParams<T> p) {
    const int64_t e = *p.epoch;
    const int tid = threadIdx.x;
    const MailLayout &L = p.lay;
    __shared__ int32_t s_box[64][6];
    if (blockIdx.x == 0 && tid < 64) {
        // own bounds: lane k folds copy k; the butterfly leaves the result in every lane
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
        int32_t *r = p.bounds_reset + (int64_t)tid * BOUND_STRIDE;
#pragma unroll
        for (int d = 0; d < 3; ++d) { r[d] = INT32_MAX; r[3 + d] = INT32_MIN; }
        if (tid < p.P && tid != p.rank) {
            int64_t *box = reinterpret_cast<int64_t *>(p.peer_mail[tid] + L.o_box) + 6 * p.rank;
#pragma unroll
            for (int d = 0; d < 6; ++d) store_sys(box + d, (int64_t)pack_epoch(e, b[d]));
        }
    }
    const int64_t *box_in = reinterpret_cast<const int64_t *>(p.mail + L.o_box);
    wait_peers(p.P, p.rank, e, p.timeout_ticks, p.ins.err, [&](int q) {
        int64_t lo = INT64_MAX;
#pragma unroll
        for (int d = 0; d < 6; ++d) {
            const int64_t w = (int64_t)((uint64_t)load_sys(box_in + 6 * q + d) >> 32);
            lo = w < lo ? w : lo;
        }
        return lo;
    });
    if (tid < 64 && tid < p.P && tid != p.rank)
#pragma unroll
        for (int d = 0; d < 6; ++d) s_box[tid][d] = (int32_t)(uint32_t)load_sys(box_in + 6 * tid + d);
    __syncthreads();

    const int64_t l = (int64_t)blockIdx.x * 256 + tid;
    const bool active = l < p.n_local;
    int32_t cx = 0, cy = 0, cz = 0;
    Snap<T> s{};
    bool ok = false, box = false;
    if (active) {
        s = p.dst[p.lo + l];
        ok = cell_of(s.x, s.y, s.z, p.ins.grid.inv_cs, cx, cy, cz);   // else: ERR_DOMAIN raised by the step
        box = p.quat && p.ins.kind[p.lo + l] != 0;
    }
    const uint64_t lt = (1ull << (tid & 63)) - 1ull;
    bool pushed = false;                          // wave-uniform
    for (int q = 0; q < p.P; ++q) {
        if (q == p.rank) continue;
        const int32_t *b = s_box[q];
        // empty bounds (min > max): the peer owns no body, needs none.
        // Compared in int64: min - 1 / max + 1 cannot overflow.
        const bool in = ok && b[0] <= b[3] && (int64_t)cx >= (int64_t)b[0] - 1 && (int64_t)cx <= (int64_t)b[3] + 1 &&
                        (int64_t)cy >= (int64_t)b[1] - 1 && (int64_t)cy <= (int64_t)b[4] + 1 &&
                        (int64_t)cz >= (int64_t)b[2] - 1 && (int64_t)cz <= (int64_t)b[5] + 1;
        const uint64_t m = __ballot(in);
        if (m == 0) continue;
        pushed = true;
        const int leader = __builtin_ctzll(m);
        int32_t base = 0;
        if ((tid & 63) == leader) base = atomicAdd(p.push_cnt + q, __popcll(m));
        base = __shfl(base, leader);
        if (in) {
            const int64_t slot = base + __popcll(m & lt);
            if (slot < p.S) {       // a peer holds at most S of this rank's bodies
                char *mail = p.peer_mail[q];
                uint32_t *ids = reinterpret_cast<uint32_t *>(mail + L.o_ids) + (int64_t)p.rank * p.S;
                Snap<T> *sn = reinterpret_cast<Snap<T> *>(mail + L.o_snap) + (int64_t)p.rank * p.S;
                __hip_atomic_store(ids + slot, (uint32_t)(p.lo + l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                store_snap_sys(sn + slot, s);
                if (box) {                        // a box: its orientation too
                    T *qm = reinterpret_cast<T *>(mail + L.o_quat) + 4 * ((int64_t)p.rank * p.S + slot);
                    const T *qs = p.quat + 4 * (p.lo + l);
#pragma unroll
                    for (int k = 0; k < 4; ++k) __hip_atomic_store(qm + k, qs[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    // the pushes are complete (acknowledged by the peer's memory) before
    // this kernel is, so before the insert kernel publishes their count
    if (pushed) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): no cache writeback needed
}

template <typename T>
__global__ __launch_bounds__(256) void halo_insert_kernel(HaloParams<T> p) {
    const int64_t e = *p.epoch;
    const int tid = threadIdx.x;
    const MailLayout &L = p.lay;
    __shared__ int64_t s_off[65];
    if (blockIdx.x == 0 && tid < p.P && tid != p.rank) {
        const int32_t n = p.push_cnt[tid];
        int64_t *cnt = reinterpret_cast<int64_t *>(p.peer_mail[tid] + L.o_cnt) + p.rank;
        store_sys(cnt, (int64_t)pack_epoch(e, n < p.S ? n : (int32_t)p.S));
        p.push_cnt[tid] = 0;
    }
    const int64_t *cnt_in = reinterpret_cast<const int64_t *>(p.mail + L.o_cnt);
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
    const uint32_t *ids = reinterpret_cast<const uint32_t *>(p.mail + L.o_ids);
    const Snap<T> *sn = reinterpret_cast<const Snap<T> *>(p.mail + L.o_snap);
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
        if (box && p.quat) copy_quat_sys(p.quat + 4 * (int64_t)id, reinterpret_cast<const T *>(p.mail + L.o_quat) + 4 * o);
        insert_id(p.ins.grid, p.ins.tab, p.ins.err, s, id | (box ? BOX_FLAG : 0u), gen);
    }
}

// ---- sharded K-step blocks: the push (XS; rb_internal.hpp) ----------------
// Before each block launch of a sharded world (rb_xblock.hip, xs != 0):
//   1. every workgroup reduces its own bodies' x / y bounds and max |v|
//      (floats rounded outward), the last to arrive publishes the rank's
//      header, epoch-tagged, into every mailbox (its own too);
//   2. every workgroup waits for all P headers of this epoch; they give the
//      launch's speed bound V = valpha max|v| + vbeta + K |g| dt over ALL
//      ranks (so every rank bounds every body alike) and the band W;
//   3. each own body within W of a peer's bounds (both axes) goes to that
//      peer's inbox of this epoch's parity: its id, snapshot and 13 state
//      rows (system-scope stores over xGMI; a wave-aggregated slot count);
//   4. the last workgroup done pushing publishes the counts, then waits for
//      every peer's counts of this epoch: when the kernel ends, this rank's
//      inbox is complete, and the block launch never waits on a peer.
// A peer writes this rank's inbox of parity e % 2 again only in its push of
// epoch e + 2, after its block launch e + 1, which needed this rank's counts
// of epoch e + 1, published after this rank's block launch e: one inbox per
// parity suffices.  Headers and counts of epoch e are overwritten only after
// this rank's push e ended likewise.  An error anywhere (this rank's error
// word at the push, a time-out, a full inbox) goes into the header's error
// word: every rank then raises ERR_XB, and all roll the run back together.
__device__ __forceinline__ float f_down(double v) { return __double2float_rd(v); }
__device__ __forceinline__ float f_up(double v) { return __double2float_ru(v); }
__device__ __forceinline__ float f_down(float v) { return v; }
__device__ __forceinline__ float f_up(float v) { return v; }

template <typename T>
__global__ __launch_bounds__(XS_PUSH_BLOCK) void xs_push_kernel(XsPushParams<T> p) {
    constexpr int NW = XS_PUSH_BLOCK / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const MailLayout &L = p.lay;
    const int64_t e = *p.xs_epoch + 1;
    const int par = (int)(e & 1);
    const unsigned nb = gridDim.x;
    __shared__ float s_red[NW][6];
    __shared__ float s_hdr[64][6];
    __shared__ int s_last;

    // 1. own partials: x min, x max, y min, y max, max |v|, error
    const int64_t l = (int64_t)blockIdx.x * XS_PUSH_BLOCK + tid;
    const bool act = l < p.n_local;
    Snap<T> s{};
    T vx = T(0), vy = T(0), vz = T(0);
    if (act) {
        s = p.snap[p.lo + l];
        vx = p.st.vx()[l]; vy = p.st.vy()[l]; vz = p.st.vz()[l];
    }
    const T sp = sqroot(vx * vx + vy * vy + vz * vz);
    const bool bad = act && !(s.x == s.x && s.y == s.y && sp == sp && fabs(s.x) < T(1e30) && fabs(s.y) < T(1e30) &&
                              sp < T(1e30));
    float b[6] = {act && !bad ? f_down(s.x) : INFINITY, act && !bad ? f_up(s.x) : -INFINITY,
                  act && !bad ? f_down(s.y) : INFINITY, act && !bad ? f_up(s.y) : -INFINITY,
                  act && !bad ? f_up(sp) : 0.f, bad ? 1.f : 0.f};
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        b[0] = fminf(b[0], __shfl_xor(b[0], off)); b[1] = fmaxf(b[1], __shfl_xor(b[1], off));
        b[2] = fminf(b[2], __shfl_xor(b[2], off)); b[3] = fmaxf(b[3], __shfl_xor(b[3], off));
        b[4] = fmaxf(b[4], __shfl_xor(b[4], off)); b[5] = fmaxf(b[5], __shfl_xor(b[5], off));
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) s_red[wave][k] = b[k];
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < NW; ++w) {
            b[0] = fminf(b[0], s_red[w][0]); b[1] = fmaxf(b[1], s_red[w][1]);
            b[2] = fminf(b[2], s_red[w][2]); b[3] = fmaxf(b[3], s_red[w][3]);
            b[4] = fmaxf(b[4], s_red[w][4]); b[5] = fmaxf(b[5], s_red[w][5]);
        }
        uint32_t *pp = reinterpret_cast<uint32_t *>(p.part) + 8 * (int64_t)blockIdx.x;
#pragma unroll
        for (int k = 0; k < 6; ++k) __hip_atomic_store(pp + k, __float_as_uint(b[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long old = __hip_atomic_fetch_add(p.done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old % nb == nb - 1) {
            // the last partial: the rank's header, to every mailbox
            float h[6] = {INFINITY, -INFINITY, INFINITY, -INFINITY, 0.f, 0.f};
            for (unsigned k = 0; k < nb; ++k) {
                const uint32_t *q = reinterpret_cast<const uint32_t *>(p.part) + 8 * (int64_t)k;
                float v[6];
#pragma unroll
                for (int j = 0; j < 6; ++j) v[j] = __uint_as_float(__hip_atomic_load(q + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                h[0] = fminf(h[0], v[0]); h[1] = fmaxf(h[1], v[1]); h[2] = fminf(h[2], v[2]);
                h[3] = fmaxf(h[3], v[3]); h[4] = fmaxf(h[4], v[4]); h[5] = fmaxf(h[5], v[5]);
            }
            if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) h[5] = 1.f;
            for (int q = 0; q < p.P; ++q) {
                int64_t *hw = reinterpret_cast<int64_t *>(p.peer_mail[q] + L.o_xhdr) + (int64_t)XS_HDR_WORDS * p.rank;
#pragma unroll
                for (int j = 0; j < XS_HDR_WORDS; ++j) store_sys(hw + j, (int64_t)pack_epoch(e, (int32_t)__float_as_uint(h[j])));
            }
        }
    }
    // 2. every rank's header of this epoch
    const int64_t *hin = reinterpret_cast<const int64_t *>(p.mail + L.o_xhdr);
    const int nw = p.P * XS_HDR_WORDS;
    int late = 0;
    for (int k = tid; k < nw; k += XS_PUSH_BLOCK) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const int64_t wd = load_sys(hin + k);
            if ((int64_t)((uint64_t)wd >> 32) >= e) {
                if ((int64_t)((uint64_t)wd >> 32) != e) late = 1;
                s_hdr[k / XS_HDR_WORDS][k % XS_HDR_WORDS] = __uint_as_float((uint32_t)wd);
                break;
            }
            if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > p.timeout_ticks ||
                (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ERR_EXCHANGE)) {
                late = 1;
                s_hdr[k / XS_HDR_WORDS][k % XS_HDR_WORDS] = k % XS_HDR_WORDS == 5 ? 1.f : 0.f;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (late) atomicOr(p.err, ERR_EXCHANGE | ERR_XB);
    __syncthreads();
    float vm = 0.f;
    bool any_err = false;
    for (int q = 0; q < p.P; ++q) {
        vm = fmaxf(vm, s_hdr[q][4]);
        any_err |= s_hdr[q][5] != 0.f;
    }
    const T V = p.valpha * (T)vm + p.vbeta + (T)p.K * p.gdt;
    const T W = (T)p.K * p.reach + T(2) * (T)(p.K > 0 ? p.K - 1 : 0) * V * p.dt + T(1e-3) * p.reach;
    if (blockIdx.x == 0 && tid == 0) {
        p.vw[0] = V;
        p.vw[1] = W;
        if (any_err) atomicOr(p.err, ERR_XB);
    }

    // 3. the own bodies each peer's blocks can reach
    bool pushed = false;
    if (p.K > 0 && !any_err) {
        const int64_t G = L.xg;
        const uint64_t lt = (1ull << lane) - 1ull;
        for (int q = 0; q < p.P; ++q) {
            if (q == p.rank) continue;
            const float *h = s_hdr[q];
            const bool in = act && !bad && h[0] <= h[1] && s.x >= (T)h[0] - W && s.x <= (T)h[1] + W &&
                            s.y >= (T)h[2] - W && s.y <= (T)h[3] + W;
            const uint64_t m = __ballot(in);
            if (m == 0) continue;
            pushed = true;
            const int leader = __builtin_ctzll(m);
            int32_t base = 0;
            if (lane == leader) base = atomicAdd(p.push_cnt + q, __popcll(m));
            base = __shfl(base, leader);
            if (!in) continue;
            const int64_t slot = base + __popcll(m & lt);
            if (slot >= G) { atomicOr(p.err, ERR_XB); continue; }
            char *mail = p.peer_mail[q];
            uint32_t *ids = reinterpret_cast<uint32_t *>(mail + L.o_xids) + ((int64_t)par * p.P + p.rank) * G;
            T *pay = reinterpret_cast<T *>(mail + L.o_xpay) + ((int64_t)par * p.P + p.rank) * XS_PAY * G;
            __hip_atomic_store(ids + slot, (uint32_t)(p.lo + l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pay + 0 * G + slot, s.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pay + 1 * G + slot, s.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pay + 2 * G + slot, s.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(pay + 3 * G + slot, s.r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
            for (int k = 0; k < 13; ++k)
                __hip_atomic_store(pay + (4 + k) * G + slot, p.st.row(k)[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // 4. the pushes are complete (acknowledged by the peers' memory); the
    // last workgroup publishes the counts and waits for the peers'
    if (pushed) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    __syncthreads();
    if (tid == 0) {
        const unsigned long long old = __hip_atomic_fetch_add(p.done + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old % nb == nb - 1;
        if (s_last) {
            for (int q = 0; q < p.P; ++q) {
                if (q == p.rank) continue;
                const int32_t n = __hip_atomic_load(p.push_cnt + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(p.push_cnt + q, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                int64_t *cw = reinterpret_cast<int64_t *>(p.peer_mail[q] + L.o_xcnt) + p.rank;
                store_sys(cw, (int64_t)pack_epoch(e, n < L.xg ? n : (int32_t)L.xg));
            }
            *p.xs_epoch = e;
        }
    }
    __syncthreads();
    if (s_last) {
        const int64_t *cin = reinterpret_cast<const int64_t *>(p.mail + L.o_xcnt);
        wait_peers(p.P, p.rank, e, p.timeout_ticks, p.err,
                   [&](int q) { return (int64_t)((uint64_t)load_sys(cin + q) >> 32); });
        if (tid < p.P) {
            int32_t n = 0;
            if (tid != p.rank) {
                const int64_t wd = load_sys(cin + tid);
                if ((int64_t)((uint64_t)wd >> 32) == e) n = (int32_t)(uint32_t)wd;
                else atomicOr(p.err, ERR_XB);
            }
            p.in_cnt[tid] = n;
        }
    }
}

template <typename T> hipError_t launch_xs_push(const XsPushParams<T> &p, hipStream_t s) {
    if (p.P < 1 || p.P > 64 || p.P * XS_HDR_WORDS > 64 * 6 || p.lay.o_xhdr < 0) return hipErrorInvalidValue;
    const int64_t nb = (p.n_local + XS_PUSH_BLOCK - 1) / XS_PUSH_BLOCK;
    hipLaunchKernelGGL((xs_push_kernel<T>), dim3((unsigned)(nb > 0 ? nb : 1)), dim3(XS_PUSH_BLOCK), 0, s, p);
    return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(256) void xs_gather_kernel(Snap<T> *dst, const Snap<T> *const *peer_snap, int32_t rank,
                                                       int64_t S, int64_t N) {
    const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= N) return;
    const int64_t q = id / S;
    if (q == rank) return;
    dst[id] = load_snap_sys(peer_snap[q] + id);
}

template <typename T> hipError_t launch_xs_gather(Snap<T> *dst, const Snap<T> *const *peer_snap, int32_t rank,
                                                  int32_t P, int64_t S, int64_t N, hipStream_t s) {
    if (P < 1 || S <= 0 || N <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL((xs_gather_kernel<T>), dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, dst, peer_snap, rank, S, N);
    return hipGetLastError();
}

template <typename T> hipError_t launch_halo_exchange(const HaloParams<T> &p, hipStream_t s) {
    if (p.P < 1 || p.P > 64 || p.S <= 0) return hipErrorInvalidValue;
    const int64_t pb = (p.n_local + 255) / 256;
    hipLaunchKernelGGL((halo_push_kernel<T>), dim3((unsigned)(pb > 0 ? pb : 1)), dim3(256), 0, s, p);
    int64_t ib = ((int64_t)(p.P - 1) * p.S + 255) / 256;
    ib = ib < 1 ? 1 : ib > 256 ? 256 : ib;
    hipLaunchKernelGGL((halo_insert_kernel<T>), dim3((unsigned)ib), dim3(256), 0, s, p);
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
template hipError_t launch_xs_push<double>(const XsPushParams<double> &, hipStream_t);
template hipError_t launch_xs_push<float>(const XsPushParams<float> &, hipStream_t);
template hipError_t launch_xs_gather<double>(Snap<double> *, const Snap<double> *const *, int32_t, int32_t, int64_t, int64_t, hipStream_t);
template hipError_t launch_xs_gather<float>(Snap<float> *, const Snap<float> *const *, int32_t, int32_t, int64_t, int64_t, hipStream_t);

}  // namespace rb
