// rb_halo.hpp — system-scope word accesses of the peer-to-peer exchanges and
// the halo push the step kernels run (rb_kernels.hip; the insert and prime
// kernels are in rb_p2p.hip).  Not part of the public interface.
#pragma once

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

__device__ __forceinline__ uint64_t pack_epoch(int64_t e, int32_t v) {
    return ((uint64_t)e << 32) | (uint32_t)v;
}

// The peers' cell bounds for this step's push, lane q holding peer q's
// (b[0..2] min, b[3..5] max; lanes of no peer: empty, min > max).  Every lane
// of the wave calls it.  They are the bounds the peer's insert (or prime)
// kernel published after the step before this one, tagged with that epoch
// + 1 (or a newer one: a peer may be a step ahead; the push margin covers
// both).  Bounded wait: after timeout_ticks (or once any exchange timed out)
// ERR_EXCHANGE is raised and false returned (nothing is pushed).  e =
// *p.halo.halo_e, loaded by the caller early in the kernel (its latency
// then hides under the step).
template <typename T>
__device__ __forceinline__ bool halo_bounds(const StepParams<T> &p, int64_t e, int32_t (&b)[6]) {
    const HaloPush &h = p.halo;
    const int lane = (int)(threadIdx.x & 63);
    const int64_t *box_in = reinterpret_cast<const int64_t *>(h.mail + h.lay.o_box);
    const bool need = lane < h.P && lane != h.rank;
#pragma unroll
    for (int d = 0; d < 3; ++d) { b[d] = 1; b[3 + d] = 0; }
    uint64_t t0 = 0;
    for (int spin = 0;; ++spin) {
        bool ok = true;
        if (need) {
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                const uint64_t w = (uint64_t)load_sys(box_in + 6 * lane + d);
                ok &= (int64_t)(w >> 32) >= e + 1;
                b[d] = (int32_t)(uint32_t)w;
            }
        }
        if (__all(ok)) return true;
        if (spin == 0) t0 = __builtin_amdgcn_s_memrealtime();
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > h.timeout_ticks ||
            (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ERR_EXCHANGE)) {
            if (lane == 0) atomicOr(p.err, ERR_EXCHANGE);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// The push of one wave's bodies (every lane calls it; a lane with a body
// passes have, its global id i and cell[0..2] its new cell, cell[3..5] its
// step-start cell; e and b as for halo_bounds).  Exact: a partner of a peer body
// lies within one cell of it (cells are >= 2 x the reach), the peer body
// lies within one cell of its step-start cell (the check below, on the
// peer's side), which lies inside the bounds read: so every body the peer's
// next search can reach lies within two cells of those bounds.  A body that
// moved more than a cell raises ERR_HALO_MOVE (the run is reported failed).
template <typename T>
__device__ __forceinline__ void halo_push(const StepParams<T> &p, int64_t e, bool have, int32_t i, const int32_t *cell,
                                          const int32_t (&b)[6]) {
    const HaloPush &h = p.halo;
    const int lane = (int)(threadIdx.x & 63);
    if (have && (abs(cell[0] - cell[3]) > 1 || abs(cell[1] - cell[4]) > 1 || abs(cell[2] - cell[5]) > 1))
        atomicOr(p.err, ERR_HALO_MOVE);
    const int par = (int)((e + 1) & 1);               // the inbox the peer's next insert reads
    const uint64_t lt = (1ull << lane) - 1ull;
    bool pushed = false;                              // wave-uniform
    for (int q = 0; q < h.P; ++q) {
        if (q == h.rank) continue;
        int32_t bq[6];
#pragma unroll
        for (int d = 0; d < 6; ++d) bq[d] = __builtin_amdgcn_readlane(b[d], q);
        // empty bounds (min > max): the peer owns no body.  int64: no overflow at +-2
        const bool in = have && bq[0] <= bq[3] && (int64_t)cell[0] >= (int64_t)bq[0] - 2 &&
                        (int64_t)cell[0] <= (int64_t)bq[3] + 2 && (int64_t)cell[1] >= (int64_t)bq[1] - 2 &&
                        (int64_t)cell[1] <= (int64_t)bq[4] + 2 && (int64_t)cell[2] >= (int64_t)bq[2] - 2 &&
                        (int64_t)cell[2] <= (int64_t)bq[5] + 2;
        const uint64_t m = __ballot(in);
        if (m == 0) continue;
        pushed = true;
        const int leader = __builtin_ctzll(m);
        int32_t base = 0;
        if (lane == leader) base = atomicAdd(h.push_cnt + q, __popcll(m));
        base = __shfl(base, leader);
        if (in) {
            const int64_t slot = base + __popcll(m & lt);
            if (slot < h.S) {                         // (a rank owns at most S bodies: always)
                char *mail = h.peer_mail[q];
                const int64_t o = (int64_t)h.rank * h.S + slot;
                __hip_atomic_store(reinterpret_cast<uint32_t *>(mail + h.lay.o_ids[par]) + o, (uint32_t)i,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                // the own new snapshot row (this lane stored it)
                store_snap_sys(reinterpret_cast<Snap<T> *>(mail + h.lay.o_snap[par]) + o, p.snap_next[i]);
                if (p.quat_next && p.cs.kind[i] != 0) {   // a box: its new orientation too
                    T *qm = reinterpret_cast<T *>(mail + h.lay.o_quat[par]) + 4 * o;
                    const T *qs = p.quat_next + 4 * (int64_t)i;
#pragma unroll
                    for (int k = 0; k < 4; ++k) __hip_atomic_store(qm + k, qs[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    // the pushes are complete (acknowledged by the peer's memory) before this
    // kernel is, so before the insert kernel publishes their count
    if (pushed) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): no cache writeback needed
}

}  // namespace rb
