// rb_internal.hpp — shared between the kernels (rb_kernels.hip) and the
// C-ABI implementation (rb_capi.hip).  Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rb {

// error bits accumulated in the world's device error word
enum : int32_t {
    ERR_BUCKET_OVERFLOW = 1,    // broadphase bucket capacity exceeded
    ERR_PARTNER_OVERFLOW = 2,   // more sphere partners than max_partners
    ERR_UNSUPPORTED = 4,        // box-involved body pair within bounding distance
    ERR_DOMAIN = 8,             // non-finite / out-of-range position
};

// Broadphase bucket entry: a snapshot of a body's step-start position plus
// what a candidate test needs (bounding radius == sphere radius for spheres,
// body kind), so the query reads nothing else by body id.
template <typename T> struct Entry;
template <> struct alignas(16) Entry<double> { double x, y, z, r; int32_t id, kind; int32_t pad[2]; };
template <> struct alignas(16) Entry<float> { float x, y, z, r; int32_t id, kind; int32_t pad[2]; };

constexpr int MAX_PLANES = 8;

// Structure-of-arrays body state.  Positions live in the replicated
// [P][3][S] buffer (this rank's slice = px/py/pz); the rest is per shard.
template <typename T> struct BodyState {
    T *px, *py, *pz;
    T *qw, *qx, *qy, *qz;
    T *vx, *vy, *vz;
    T *wx, *wy, *wz;
};

// Per-body constants, global body index (replicated on every rank).
template <typename T> struct BodyConsts {
    const T *mass, *ix, *iy, *iz;      // principal inertia (body frame)
    const T *sx, *sy, *sz;             // sphere radius / box half extents
    const T *bound;                    // bounding-sphere radius
    const int32_t *kind;
};

template <typename T> struct Grid {
    T inv_cs;                          // 1 / cell size
    uint32_t hmask;                    // H - 1 (H power of two)
    int32_t cap;                       // entries per bucket
    int32_t H;
};

template <typename T> struct StepParams {
    int64_t n_global;
    int32_t n_local, lo;
    BodyState<T> st;
    BodyConsts<T> cs;
    const T *xfrc;                     // [6][S] or nullptr
    int32_t S;
    int32_t n_planes;
    T pn[MAX_PLANES][3], pp[MAX_PLANES][3];
    T g[3];
    T dt, e, mu, thr;
    int32_t oriented;
    Grid<T> grid;
    const int32_t *cnt_cur;
    const Entry<T> *ent_cur;
    int32_t *cnt_next;
    Entry<T> *ent_next;
    int32_t *cnt_clear;
    int32_t *err;
    // optional contact recording ([n_local][maxrec] slots)
    int32_t *rec_count, *rec_partner, *rec_kind;
    T *rec_dist;
    int32_t maxrec;
};

template <typename T> struct InsertParams {
    const T *gpos;                     // [P][3][S]
    const T *bound;                    // [Npad] bounding radius
    const int32_t *kind;               // [Npad]
    int32_t S;
    int64_t first, count;              // global ids [first, first+count)
    int64_t skip_lo, skip_hi;          // global ids to skip (already inserted)
    Grid<T> grid;
    int32_t *cnt;
    Entry<T> *ent;
    int32_t *err;
};

// launchers (rb_kernels.hip)
template <typename T> hipError_t launch_step(const StepParams<T> &p, int maxp, bool coop, hipStream_t s);
template <typename T> hipError_t launch_insert(const InsertParams<T> &p, hipStream_t s);
template <typename T> hipError_t launch_kat_impulse(int64_t n, const double *in, double *out, hipStream_t s);
template <typename T> hipError_t launch_kat_inertia(int64_t n, const double *in, double *out, hipStream_t s);
template <typename T> hipError_t launch_kat_apply(int64_t n, const double *in, double *out, hipStream_t s);

constexpr int STEP_BLOCK = 64;

}  // namespace rb
