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
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const int64_t id = (int64_t)blockIdx.x * 256 + tid;
    if (id >= p.ins.count || (id >= p.ins.skip_lo && id < p.ins.skip_hi)) return;
    const Snap<T> s = p.peer_snap[id / p.S][id];
    p.dst[id] = s;
    insert_id(p.ins.grid, p.ins.tab, p.ins.err, s, (uint32_t)id | (p.ins.kind[id] != 0 ? BOX_FLAG : 0u));
}

template <typename T> hipError_t launch_p2p_exchange(const P2PParams<T> &p, hipStream_t s) {
    if (p.ins.count <= 0 || p.P < 1 || p.P > 64) return hipErrorInvalidValue;
    const int64_t blocks = (p.ins.count + 255) / 256;
    hipLaunchKernelGGL((p2p_exchange_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t launch_p2p_exchange<double>(const P2PParams<double> &, hipStream_t);
template hipError_t launch_p2p_exchange<float>(const P2PParams<float> &, hipStream_t);

}  // namespace rb
