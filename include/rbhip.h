/*
 * rbhip.h — C-ABI of librbhip.so, the MI355X-native (gfx950) many-body
 * rigid-body stepper that sits behind the src/physics / src/simulation call
 * surface of pratyay2510/RigidBody-Simulation.
 *
 * The reference has no FFI: every entry point below replaces a Python call
 * site of the reference (cited per function, paths relative to the reference
 * repository root).  The ctypes binding a maintainer would add on the
 * reference side is shown in INTEGRATION.md; the in-tree binding is
 * rigidbody-simulation_amd/rbhip/_lib.py.
 *
 * Conventions
 *   - Every function returns 0 on success or a negative errno-style code
 *     (RB_E*); rb_last_error() returns a thread-local message for the last
 *     failure on the calling thread.
 *   - Host buffers are owned by the caller and never retained past a call.
 *     Device buffers are owned by the library (a world).
 *   - A world handle is not thread-safe: one world per host thread.
 *   - Results are deterministic: independent of launch geometry, of the
 *     number of ranks a scene is sharded over, and of run-to-run scheduling.
 *   - State layout at the boundary is the reference's MuJoCo layout:
 *     qpos stride 7 (x y z qw qx qy qz), qvel stride 6 (vx vy vz wx wy wz),
 *     body k (0-based among free bodies) at qpos[7k], qvel[6k]
 *     (multi_sphere_bounce.py:50-51 with the SURVEY D1 off-by-one fixed).
 *     Inside the library the state is struct-of-arrays in HBM.
 */
#ifndef RBHIP_H
#define RBHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define RB_OK            0
#define RB_EINVAL      (-22)  /* bad argument / descriptor                      */
#define RB_ENOMEM      (-12)  /* device or host allocation failed               */
#define RB_ENODEV      (-19)  /* no HIP device / HIP runtime failure            */
#define RB_EOVERFLOW   (-75)  /* contact or broadphase-bucket capacity exceeded */
#define RB_EUNSUPPORTED (-95) /* unsupported combination (e.g. the two-ball law in a sharded world) */
#define RB_EDOM        (-33)  /* non-finite or out-of-range body position       */

/* ---- enums ------------------------------------------------------------- */
#define RB_BODY_SPHERE   0    /* size = (radius, -, -)                          */
#define RB_BODY_BOX      1    /* size = half extents (hx, hy, hz)               */

#define RB_F64           0
#define RB_F32           1

/* MuJoCo stores one normal per contact, pointing geom1 -> geom2.
 * RAW applies it unchanged to both bodies (what collision.py:27 does);
 * ORIENTED flips it for the body that is geom1 so it always points toward
 * the body being solved.  Plane contacts are identical in both modes. */
#define RB_NORMAL_ORIENTED 0
#define RB_NORMAL_RAW      1

/* contact laws (rb_set_contact_law) */
#define RB_LAW_MUJOCO    0    /* the per-body Gauss-Seidel law of collision.py / multi_sphere_bounce.py (default) */
#define RB_LAW_BALLS     1    /* the symmetric two-ball law of ball_collision.py */

/* contact kinds reported by rb_get_contacts */
#define RB_CK_PLANE_SPHERE   0
#define RB_CK_PLANE_BOX0     1   /* 1 + corner index (0..7, corner bits i&1,i&2,i&4) */
#define RB_CK_SPHERE_SPHERE 16
/* Box-involved kinds are this project's restatement of MuJoCo's sphere-box /
 * box-box primitives (not available offline): parity against MuJoCo is
 * UNPINNED (the reference's only box, models/cube.xml:35, never meets
 * another box or a sphere).  Known divergence: a face contact keeps at most
 * the 4 deepest clipped points, where mjc_BoxBox may return more and select
 * differently. */
#define RB_CK_SPHERE_BOX    17   /* sphere = geom1 (MuJoCo dispatches by geom type) */
#define RB_CK_BOX_BOX0      32   /* 32 + k: k-th face-clip point of a box pair (k < 4) */
#define RB_CK_BOX_EDGE      40   /* edge-edge point of a box pair */

/* ---- scene descriptor -------------------------------------------------- */
typedef struct rb_scene_desc {
    int64_t n_bodies;          /* global body count N                                  */
    int32_t n_planes;          /* <= RB_MAX_PLANES static half-spaces                   */
    int32_t dtype;             /* RB_F64 | RB_F32 (arithmetic type of the path)        */
    int32_t normal_convention; /* RB_NORMAL_ORIENTED | RB_NORMAL_RAW                   */
    int32_t device;            /* HIP device ordinal                                   */
    int32_t rank;              /* shard index: owns bodies [rank*S, rank*S+S) ∩ [0,N)  */
    int32_t world_size;        /* shard count P; S = ceil(N / P)                       */
    int32_t max_partners;      /* sphere-sphere contacts per body (0 = default 16; a guarded rb_step chunk raises 16 to 32 on overflow) */
    int32_t bucket_capacity;   /* reserved (0): a broadphase bucket holds 30 ids       */
    const int32_t *kind;       /* [N]   RB_BODY_*                                      */
    const double  *mass;       /* [N]   model.body_mass of each free body              */
    const double  *inertia;    /* [N*3] model.body_inertia (principal, body frame)     */
    const double  *size;       /* [N*3] sphere: (r, 0, 0); box: half extents           */
    const double  *planes;     /* [n_planes*6] (normal xyz, point xyz), world frame    */
    double         gravity[3]; /* model.opt.gravity                                    */
} rb_scene_desc;

#define RB_MAX_PLANES 8

typedef struct rb_world rb_world;

/* ---- lifetime ---------------------------------------------------------- */
/* Replaces the MjModel/MjData pair the reference step functions receive
 * (collision.py:56, time_integeration.py:13, multi_sphere_bounce.py:42):
 * masses, inertias, geometry and gravity become explicit SoA device arrays. */
int  rb_world_create(rb_world **out, const rb_scene_desc *desc);
void rb_world_destroy(rb_world *w);
const char *rb_last_error(void);
const char *rb_version(void);

/* Bind the world to a caller-owned HIP stream (hipStream_t; NULL is HIP's
 * default null stream, e.g. torch's default stream).  Until this is called
 * the world uses a private non-blocking stream.  All later work of this
 * world is enqueued on the bound stream. */
int rb_set_stream(rb_world *w, void *hip_stream);

/* ---- state transfer (the only AoS<->SoA transposes) --------------------- */
/* Global arrays: qpos [N*7], qvel [N*6] (host).  set: every rank passes the
 * whole scene; the world keeps all positions and its own shard of the rest.
 * get: writes the rows of the bodies this world owns, leaves others alone.
 * Replaces the reads/writes of data.qpos/data.qvel at collision.py:60-65,
 * :97-100 and multi_sphere_bounce.py:50-51, :85-88. */
int rb_set_state(rb_world *w, const double *qpos, const double *qvel);
int rb_get_state(rb_world *w, double *qpos, double *qvel);
/* optional data.xfrc_applied [N*6] (force xyz, torque xyz); NULL = zero
 * (collision.py:66-67).  Host pointer, copied. */
int rb_set_xfrc(rb_world *w, const double *xfrc);

/* ---- the hot path ------------------------------------------------------ */
/* nsteps reference steps: contact generation (mj_forward's role,
 * collision.py:57), gravity (collision.py:66-70), the per-contact
 * Gauss-Seidel impulse solve with Coulomb friction (collision.py:72-88 ->
 * compute_collision_impulse_friction collision.py:7-48 ->
 * apply_impulse_friction physics_utils.py:25-49) and the semi-implicit
 * position/quaternion integration (collision.py:90-100).  Jacobi across
 * bodies (one contact pass per step, multi_sphere_bounce.py:43-46).
 * contact_threshold: contacts with |dist| < threshold are skipped
 * (collision.py:79-80; 0 there, 1e-4 in time_integeration.py:13).
 * Synchronous: returns after the device finished, with any device-side
 * error (overflow, unsupported pair, non-finite position) reported. */
int rb_step(rb_world *w, int64_t nsteps, double dt, double restitution,
            double friction, double contact_threshold);
/* Same, enqueued only (no host sync, no error check).  rb_sync waits and
 * returns the accumulated device-side error. */
int rb_step_async(rb_world *w, int64_t nsteps, double dt, double restitution,
                  double friction, double contact_threshold);
int rb_sync(rb_world *w);

/* ---- sharded stepping (world_size > 1) ---------------------------------- */
/* One step of the owned bodies; their new positions land in this rank's
 * slice of the replicated position buffer of the next step.  The caller then
 * all-gathers that buffer (RCCL over xGMI via torch.distributed, or any
 * transport) and calls rb_shard_exchange_done, which publishes the other
 * ranks' positions to the next step's broadphase.  Both calls are enqueued
 * only. */
int rb_shard_step(rb_world *w, double dt, double restitution, double friction,
                  double contact_threshold);
int rb_shard_exchange_done(rb_world *w);
/* Device view of the position buffer the pending exchange fills (valid
 * between rb_shard_step and rb_shard_exchange_done; two buffers alternate
 * step by step).  Layout [P][S][4] of the world's dtype — (x, y, z,
 * bounding radius) per body, bodies in global id order; this rank's slice
 * is the contiguous [rank][S][4] (shard_elems = 4*S elements). */
int rb_gpos_buffer(rb_world *w, void **dev_ptr, int64_t *shard_elems,
                   int32_t *elem_bytes);
/* Worlds with box bodies: the orientation buffer the same exchange fills
 * alongside (layout [P][S][4], (w, x, y, z) per body in global id order, rows
 * of box bodies meaningful) — all-gather it like the position buffer.  A
 * sphere-only world returns *dev_ptr = NULL and *shard_elems = 0 (nothing
 * to exchange: a sphere's contacts never read its orientation).  No reference
 * counterpart (the reference is single-process; its box body is
 * models/cube.xml:35). */
int rb_gquat_buffer(rb_world *w, void **dev_ptr, int64_t *shard_elems,
                    int32_t *elem_bytes);

/* In-library exchange: the library owns an RCCL communicator over the
 * world's ranks (RCCL is loaded at first use; the single-GPU path never
 * needs it) and runs the per-step exchange itself, so K sharded steps --
 * step kernel, in-place all-gather of the position buffer over xGMI, remote
 * insert -- replay from one captured HIP graph with no host work per step.
 * Replaces the per-frame loop of custom_step_multi_sphere
 * (multi_sphere_bounce.py:42-92) on a body-range sharded scene.
 *   rb_comm_unique_id: rank 0 creates the communicator id (bytes >= 128)
 *     and hands it to every rank (e.g. torch.distributed broadcast);
 *   rb_shard_comm_init: every rank joins (blocks until all have); the
 *     world's device, rank and world_size define the communicator;
 *   rb_shard_run: nsteps sharded steps, enqueued only; every rank must make
 *     the same calls with the same nsteps.  Bit-identical to rb_shard_step +
 *     all-gather + rb_shard_exchange_done, and to rb_step for world_size 1. */
int rb_comm_unique_id(void *id, int32_t bytes);
int rb_shard_comm_init(rb_world *w, const void *id, int32_t bytes);
int rb_shard_run(rb_world *w, int64_t nsteps, double dt, double restitution,
                 double friction, double contact_threshold);

/* Peer-to-peer exchange (SURVEY §7 hard part 4), in place of the RCCL
 * all-gather: after its step kernel each rank flags "step done" into every
 * peer's flag word, and its exchange kernel reads the other ranks' fresh
 * slices straight from their buffers over xGMI (IPC mappings) once they
 * have flagged, then inserts them.  Waits are bounded: a peer missing for
 * 5 s raises RB_ENODEV at the next rb_sync instead of hanging.
 *   rb_p2p_handles: this rank's IPC handles (*len bytes; out = NULL to ask
 *     the size); every rank passes the concatenation of all ranks' handles,
 *     in rank order, to
 *   rb_p2p_connect (collective: no rank may step before all have connected).
 * rb_shard_run then uses this transport; bit-identical to the others. */
int rb_p2p_handles(rb_world *w, void *out, int64_t cap, int64_t *len);
int rb_p2p_connect(rb_world *w, const void *all, int64_t len);

/* Halo mode of the peer-to-peer exchange, for large shards (no reference
 * counterpart: the reference is single-process).  Instead of reading every
 * peer's whole slice, the step kernel of each rank pushes to each peer only
 * its bodies whose new cell lies within two cells of that peer's own
 * bodies' cell bounds of the step before (a superset of everything the
 * peer's next contact searches can reach while no body moves more than one
 * broadphase cell per step; one that does fails the run with RB_EDOM), into
 * the peer's inbox; one insert kernel per step then publishes the bounds
 * and counts and inserts what the peers pushed.  No host work; still
 * bit-identical to every other transport.  Collective: every rank must make
 * the same call, after rb_p2p_connect and before stepping.  enable = 0
 * returns to full reads. */
int rb_p2p_halo(rb_world *w, int32_t enable);

/* ---- the two-ball law -------------------------------------------------- */
/* Switch a world to RB_LAW_BALLS (or back to RB_LAW_MUJOCO), replacing
 * step_with_custom_collisions (ball_collision.py:73-125): gravity v += g dt;
 * ground contact against z = 0 when z < r (impulse, then z = r); ball-ball
 * contact when |p_b - p_a| < r_a + r_b + tol with the full-effective-mass
 * impulse compute_collision_impulse (ball_collision.py:53-68) and half-overlap
 * position correction; x += v dt; quaternions untouched.  Two balls step
 * exactly as the reference; N balls evaluate every pair from the post-ground
 * state of both and accumulate per ball in ascending partner id.  Requires
 * spheres only, world_size 1, and either no plane or exactly the ground
 * plane (normal (0,0,1) through the origin); tol >= 0 (the reference: 0.01).
 * rb_step's contact_threshold is ignored under this law. */
int rb_set_contact_law(rb_world *w, int32_t law, double tol);

/* ---- parity support ---------------------------------------------------- */
/* Record the contact list generated during the most recent step (off by
 * default: recording costs HBM traffic).  Canonical per-body order: plane
 * contacts (plane order; box corners in bit order), then partners by
 * ascending body id (a box-involved partner: its contacts in generation
 * order, RB_CK_SPHERE_BOX / RB_CK_BOX_BOX0 + k / RB_CK_BOX_EDGE), in
 * sharded worlds as well (their exchange carries the boxes' orientations:
 * rb_gquat_buffer).  Output is CSR over the owned bodies: counts[n_owned];
 * partner (body id, or -1-plane_index), kind (RB_CK_*), dist.  cap is the
 * capacity of the flat arrays; total receives the number of records. */
int rb_record_contacts(rb_world *w, int enable);
int rb_get_contacts(rb_world *w, int32_t *counts, int32_t *partner,
                    int32_t *kind, double *dist, int64_t cap, int64_t *total);

/* Known-answer entries, run as device kernels on `device`.
 * rb_kat_impulse: per case in[24] = m, e, mu, v[3], w[3], r[3], n[3],
 * inertia_world[9] (row-major) -> out[10] = jn, jt[3], v'[3], w'[3]:
 * compute_collision_impulse_friction (collision.py:7-48) followed by
 * apply_impulse_friction (physics_utils.py:25-49).  dtype RB_F64|RB_F32.
 * rb_kat_inertia: per case in[7] = inertia_diag[3], q[4] (wxyz) ->
 * out[18] = inertia_world[9], inv(inertia_world)[9]
 * (compute_inertia_tensor_world collision.py:51-53 + np.linalg.inv). */
int rb_kat_impulse(int32_t device, int32_t dtype, int64_t n, const double *in,
                   double *out);
int rb_kat_inertia(int32_t device, int32_t dtype, int64_t n, const double *in,
                   double *out);
/* rb_kat_pair_impulse: per case in[27] = m, e, mu, v[3], w[3], r[3], n[3],
 * I_inv[9] (row-major) -> out[3] = impulse: compute_collision_impulse
 * (ball_collision.py:53-68). */
int rb_kat_pair_impulse(int32_t device, int32_t dtype, int64_t n, const double *in,
                        double *out);
/* rb_kat_narrow: the box-involved narrowphase (this
 * project's restatement of MuJoCo's sphere-box / box-box primitives, which
 * are not available offline — parity against MuJoCo is unpinned):
 * per case in[22] = kind1, kind2 (RB_BODY_*), c1[3], q1[4] (wxyz), size1[3],
 * c2[3], q2[4], size2[3] (body 1 = the lower id) -> out[33] = count, then
 * per contact dist, pos[3], frame[3] (geom1 -> geom2; a sphere is geom1 of
 * a sphere-box pair), kind (RB_CK_*). */
int rb_kat_narrow(int32_t device, int32_t dtype, int64_t n, const double *in, double *out);
/* rb_kat_apply: apply_impulse_friction alone (physics_utils.py:25-49) with
 * caller-given impulses: in[26] = m, v[3], w[3], r[3], n[3], jn, jt[3],
 * inertia_world[9] -> out[6] = v'[3], w'[3]. */
int rb_kat_apply(int32_t device, int32_t dtype, int64_t n, const double *in,
                 double *out);

/* Introspection for measurement: per-body algorithmic HBM bytes of one
 * step (state read+write + constants), number of owned bodies, and the
 * average device duration (ms) of the step kernel over the launches timed
 * since the last reset (HIP events on the world's stream; enable first). */
int rb_query(rb_world *w, int64_t *n_owned, int64_t *bytes_per_body_step);

/* Counters for tests and measurement; fills out[0 .. min(n, RB_STATS_COUNT))
 * and returns how many.
 * ABI note: librbhip 0.3 (rb_version) renumbered the counters of 0.2 — the
 * round-4 block counters were removed and RB_STAT_FORM, _BUCKETS,
 * _MAX_PARTNERS and _IO_* moved (8 -> 1, 19 -> 6, 20 -> 7, 27/28 -> 8/9;
 * RB_STATS_COUNT 30 -> 18, then 19 with RB_STAT_HASHED_FORM appended).  A
 * consumer built against the 0.2 header must be rebuilt; from 0.3 on new
 * counters are only appended. */
#define RB_STAT_GRAPHS          0   /* captured step graphs alive               */
#define RB_STAT_FORM            1   /* step kernel form of the next run: 0 one-lane, 1 cooperative, 2 wide,
                                       3 cooperative + helper, 4 wide + helper (hashed cells),
                                       5 cell-ordered tiles (rb_tiles.hip) */
#define RB_STAT_BOX_OPT         2   /* box worlds: chunks replayed without the box kernel */
#define RB_STAT_BOX_ROLLBACK    3   /* of which rolled back and replayed with it (a body was deferred) */
#define RB_STAT_REFITS          4   /* broadphase layout refits of a drifting scene (chunk rolled back, replayed) */
#define RB_STAT_TABLE_GROWS     5   /* of which with the bucket table doubled */
#define RB_STAT_BUCKETS         6   /* buckets per table now */
#define RB_STAT_MAX_PARTNERS    7   /* max_partners now (16 -> 32 after an overflow in a guarded chunk) */
#define RB_STAT_IO_SKIPPED      8   /* rb_set_state calls that were no-ops (the bytes rb_get_state handed out) */
#define RB_STAT_IO_UPLOADS      9   /* rb_set_state calls that uploaded          */
#define RB_STAT_TILE_RUNS      10   /* runs stepped in the cell-ordered tile form */
#define RB_STAT_TILE_STEPS     11   /* steps of those runs committed (checked)  */
#define RB_STAT_TILE_ROLLBACKS 12   /* tile runs rolled back and replayed by the hashed-cell forms */
#define RB_STAT_TILE_BUILDS    13   /* tile bins built from the id-ordered state */
#define RB_STAT_TILE_WHY       14   /* why bits of the rolled-back tile runs (OR; 1 bin capacity, 2 window
                                       capacity, 4 far list, 8 partners, 16 position) */
#define RB_STAT_TILE_SLOTS     15   /* tile slots of the periodic tile grid (workgroups per step) */
#define RB_STAT_TILE_COLS      16   /* columns per tile edge                    */
#define RB_STAT_TILE_ON        17   /* the next run of >= 2 steps would use the tile form */
#define RB_STAT_HASHED_FORM    18   /* the hashed-cell form (0-4, as RB_STAT_FORM) the world steps with when
                                       the tile form does not */
#define RB_STATS_COUNT         19
int rb_world_stats(rb_world *w, int64_t *out, int32_t n);
int rb_kernel_timing(rb_world *w, int enable, double *avg_ms, int64_t *launches);

/* Retired (kept for ABI compatibility with librbhip 0.2): the round-3 tile
 * blocks' configuration.  mode -1 (auto) and 0 (off) are accepted and do
 * nothing; mode 1 returns RB_EUNSUPPORTED.  The step forms are chosen by the
 * library (RB_STAT_FORM); RBHIP_TILE selects the tile form for tests. */
int rb_tile_config(rb_world *w, int32_t mode, int32_t kmax, double band, int64_t owned);

#ifdef __cplusplus
}
#endif
#endif /* RBHIP_H */
