// ctx.h — the context of the fused C ABI (include/iblb.h part 2) and the host helpers shared by
// its translation units:
//   iblb_ctx.hip   lifecycle, state, Lagrangian points, readers, checkpoint / restart
//   ctx_step.hip   halo exchange, the one-step / two-step / deep schedules, iblb_step, local and
//                  RCCL groups, the output gather
//   ctx_band.hip   the IB band cycle (K iterations per cycle with an owed force every iteration)
//
// Time-step bookkeeping.  The reference iteration (main.cu:852-909) is
//   f0,F = equilibrium(u^t, rho^t, force^t); f1 = collision(f^t); f^{t+1} = stream(f1);
//   rho^{t+1}, u_raw = macro(f^{t+1}); F_s = interpolate(...); force^{t+1}, u^{t+1} = spread(...)
// The context stores g = f1^{t-1} (post-collision, not yet streamed).  One fused launch pulls f^t
// from g, recomputes rho^t and u^t = (sum c f + force^t/2)/rho^t, collides and stores f1^t.
// force^t (the IB part of the PREVIOUS reference iteration) is computed lazily just before it is
// needed — before the next collide, before a reader, or before the Lagrangian points change — so
// every call sees exactly the reference's state.  The flux term q(u^t) the reference adds at the
// end of iteration t-1 is added by the collide of step t; iblb_get_flux() adds the not-yet-collided
// last term on demand.
//
// Slabs and ghost columns.  A context owns the columns [x_begin, x_begin + ncol) of the lattice.
// Every population buffer holds `gc` ghost columns on each side of them (columns -gc .. -1 and
// ncol .. ncol+gc-1 of the same interleaved layout, contiguous with the slab's own columns).  A
// slab of a group receives its neighbours' edge columns there — d whole columns per side, one
// contiguous block each way, sent and received by RCCL in place (no pack kernel, no slot map) —
// and every kernel reads them like its own columns.  `ghost` records how many of them hold the
// current state.  A lone slab wraps periodically inside the kernels and fills its ghosts (with
// its own edge columns) only for IB band trapezoids that cross x = 0.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <climits>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "../../include/iblb.h"

#include "cilia_kernels.h"
#include "iblb_kernels.h"

namespace iblbh {
using namespace iblb;

enum Phase { PH_EMPTY = 0, PH_BOOT = 1, PH_RUN = 2 };
enum IbState { IB_NONE = 0, IB_PENDING = 1, IB_READY = 2 };
enum Transport { TR_NONE = 0, TR_LOCAL = 1, TR_RCCL = 2 };
enum EvKind { EV_FUSED = 0, EV_IB = 1, EV_HALO = 2, EV_SWEEP = 3, EV_SWEEPK = 4 };

constexpr long GUARD = 512;  // elements in front of / behind every population buffer
constexpr int BAND_PIN_SLOTS = 4;

long env_long(const char* name, long dflt);
extern std::string g_create_error;

}  // namespace iblbh

struct iblb_ctx {
    iblb_config cfg{};
    int nx = 0, ny = 0, x_begin = 0, ncol = 0;
    int prec = IBLB_PREC_F64;
    size_t esize = 8;
    int V = 2, nch = 1;
    iblb::Layout L{};
    int gc = 0;       // ghost columns per side in every population buffer and in the dense force
    long fplane = 0;  // plane stride of the dense force and the boot fields: (ncol + 2 gc) * rows
    int device = 0;
    // kernel configuration: measured defaults; the IBLB_* knobs of INTEGRATION.md §4
    int variant = 0;            // one-step collide variant (IBLB_FUSED_VARIANT)
    bool sweep_on = true;       // multi-iteration sweeps (IBLB_SWEEP)
    int sweep_w = 4, sweep_vs = 2;  // two-iteration sweeps: columns per wave, cells per lane
    int sweep_depth = 5;        // K iterations per deep launch (IBLB_SWEEP_DEPTH; 2 = two-step only)
    int deep_w = 96, deep_vs = 2, deep_variant = 1, deep_balance = 1;  // IBLB_DEEP_W / _VS / _VARIANT / _BALANCE
    int slab_vs = 1;            // cells per lane of a group slab's deep sweeps
    int int_variant = -1;       // deep variant of a group slab's interior sweep (IBLB_INTERIOR_VARIANT; -1: deep_variant)
    int edge_trim = 0;          // slab interiors: first / last sweep narrower by this (IBLB_EDGE_TRIM)
    int reserved_cus = 0, ncu = 0;  // CUs kept free of the compute stream (RCCL groups), device CUs
    std::vector<uint32_t> comp_mask;  // the compute stream's CU mask when reserved_cus > 0
    hipStream_t stream = nullptr;
    iblb::Coef coef{};
    iblb::KConst kc{};  // collide constants folded from coef (kernel arguments)
    // populations: two buffers (ping-pong) in one allocation, each (ncol + 2 gc) columns; g[i]
    // points at column 0 of buffer i; `cur` holds the state
    char* g_alloc = nullptr;
    void* g[2] = {nullptr, nullptr};
    int cur = 0;
    long buf_elems = 0;  // elements of one buffer (ghost columns included)
    // boot arrays (slab layout, plane stride fplane)
    double* rho0 = nullptr;
    double* u0 = nullptr;
    double* force0 = nullptr;
    // immersed boundary
    int max_points = 0, ns = 0;
    bool cilia_on = false;  // on-device cilia kinematics (iblb_set_cilia)
    iblb_cilia cilia{};
    float* cil_samples = nullptr;  // the reference's d_boundary [5 * 9600 * c_num]
    float* cil_lasts = nullptr;    // [2 * 9600 * c_num]
    float* cil_bpoints = nullptr;  // [5 * 96 * c_num]
    float* d_s = nullptr;
    float* d_us = nullptr;
    float* d_Fs = nullptr;
    int* d_eps = nullptr;
    float* d_Fs_sum = nullptr;     // F_s summed over an RCCL group (reader scratch)
    std::vector<float> pts_host;   // (x, y) of the static points (band plans)
    // points given ahead (iblb_set_lagrangian_steps): entry i is used by iteration sch_t0 + i;
    // sch_cur is the entry of the current points (pts_*)
    float* d_sch_s = nullptr;
    float* d_sch_us = nullptr;
    int* d_sch_eps = nullptr;
    size_t sch_cap = 0;  // entries allocated
    int sch_n = 0, sch_cur = -1;
    long long sch_t0 = 0;
    std::vector<float> sch_x;       // [sch_n][ns][2]: (x, y) of every entry (band plans)
    std::vector<float> sch_x_prev;  // the points before the schedule (their force may be owed)
    bool cil_sched = false;         // the schedule is the cilia kinematics run ahead (cilia_schedule)
    // dense IB force [2][(ncol + 2 gc) * rows] and a flag per (column, row chunk); fdense and
    // flags point at column 0
    double* fd_alloc = nullptr;
    double* fdense = nullptr;
    uint8_t* fl_alloc = nullptr;
    uint8_t* flags = nullptr;
    // ---- IB band cycle (ctx_band.hip) ----
    int band_on = 1;             // IBLB_IB_BAND
    bool band_valid = false;     // the installed plan covers the points of the next cycle
    bool band_dirty = false;     // static points changed (or the context was linked): plan again
    std::vector<std::array<int, 4>> band_b;  // installed patches {x0, x1, y0, y1} (local columns)
    int band_d = 0;              // ghost depth the installed trapezoids read (0: all inside the slab)
    int band_x = 0;              // halo depth of the cycle's exchange (slab groups; same on every rank)
    int* band_pin[iblbh::BAND_PIN_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
    size_t band_pin_cap = 0;     // ints per slot
    hipEvent_t band_pin_ev[iblbh::BAND_PIN_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
    int band_pin_i = 0, band_pin_cur = -1;
    int* band_tab = nullptr;     // the installed plan's level tables (a pinned slot)
    std::vector<int> band_off, band_n, band_nchl;  // level j: first entry, entries, chunks per entry
    long long band_deep_lu = 0, band_lu = 0;       // cells of the deep sweep / of all trapezoid levels
    int band_flux = -1, band_fy0 = 0, band_fy1 = 0;  // flux column in a patch output, the patch's rows
    bool band_run = false;       // the last step was a band cycle on band_st / deep_st (not joined)
    long long band_retry_t = 0;  // a declined schedule plan: next attempt at this iteration
    hipEvent_t band_end = nullptr; // recorded on the deep stream at the end of the last band cycle
    char* s_alloc = nullptr;     // two scratch population buffers of the trapezoid (layout of g)
    void* sbuf[2] = {nullptr, nullptr};
    int probe_level = 0;         // timing probe IBLB_PROBE_LEVEL (lbm_kernels.hip:band_level_kernel)
    int wrap_split = 1;          // IBLB_WRAP_SPLIT: image groups of their own for points at the x edge (wrap_range)
    int band_deep_variant = -1;  // IBLB_BAND_DEEP_VARIANT: the band cycle's deep variant (-1: band_deep's choice)
    int band_merge = 1;          // IBLB_BAND_MERGE: 1 auto, 2 always, 0 never: each level's launch also
                                 // evaluates the next level's force (merged chain)
    bool band_merged = false;    // the installed plan runs the merged chain
    int band_vhalf_env = 1;      // IBLB_BAND_VHALF: f32 chained chain's level launches at half-height waves
    bool band_vhalf = false;     // the installed plan's level entries are in chunks of 64 * V/2 rows
    double* bf_alloc = nullptr;  // merged chain: two more dense force buffers (levels j % 3 = 1, 2) ...
    uint8_t* bfl_alloc = nullptr;  // ... and their chunk flags (zero between cycles)
    double* bfd[2] = {nullptr, nullptr};
    uint8_t* bfl[2] = {nullptr, nullptr};
    int band_par_env = 1;        // IBLB_BAND_PAR: the last level beside the deep sweep (lone and group slabs)
    bool band_par = false;       // the installed plan runs it (patch output rows skipped by the deep sweep)
    bool band_prev_par = false;  // the last band cycle ran it (its deep sweep ended on ev_deep)
    std::vector<iblb::SkipBox> band_skip;  // the plan's patch output regions (own columns, even rows)
    hipEvent_t ev_deep = nullptr;  // the last band cycle's deep sweep done (PAR cycles)
    int band_reserve = 0;        // CUs of the band chain's stream (0: one stream, in sequence; -2: unmasked)
    bool band_sticky = false;    // keep the streams while a schedule runs
    hipStream_t band_st = nullptr;  // the band chain (masked to the reserved CUs)
    hipStream_t deep_st = nullptr;  // the cycle's deep sweep (masked to the other CUs)
    hipEvent_t ev_b0 = nullptr, ev_bd = nullptr;
    // flux: d_Q[0] cumulative, d_Q[1] scratch
    double* d_Q = nullptr;
    // state machine
    int phase = iblbh::PH_EMPTY;
    long long t = 0;
    int ib_state = iblbh::IB_NONE;
    int ghost = 0;  // ghost columns per side holding the current state's neighbour columns
    int bnd_w = INT_MAX;  // edge columns per side the last step wrote on the comm stream
                          // (INT_MAX: the comm stream already follows the whole last step)
    // transport
    int transport = iblbh::TR_NONE;
    iblb_ctx* left = nullptr;
    iblb_ctx* right = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool self_ring = false;  // one rank that is its own neighbour over RCCL (IBLB_RCCL_SELF, rehearsal)
    std::vector<int> slab_begin, slab_count;  // every rank's columns (RCCL group)
    int min_slab = 0;                         // the narrowest slab of the group
    hipStream_t comm_stream = nullptr;  // RCCL halo exchange and boundary columns, beside the interior
    hipStream_t rccl_last = nullptr;    // the stream of the last RCCL call (ops stay in issue order)
    hipEvent_t ev_bnd = nullptr;  // comm-stream work of the last step done
    hipEvent_t ev_int = nullptr;  // compute-stream work of the last step done
    hipEvent_t ev_int2 = nullptr; // spare: a deep slab cycle's interior signals it on completion
    hipEvent_t ev_pre = nullptr;  // compute-stream work before this step
    hipEvent_t ev_x = nullptr;    // the band cycle's halo exchange done
    hipEvent_t ev_rccl = nullptr; // orders RCCL calls across streams
    bool deep_chain = false;      // the last compute work is a deep slab cycle's (interior first) ...
    long long deep_chain_t = -1;  // ... that ended at this t with this cur: ev_int follows its interior
    int deep_chain_cur = -1;
    bool overlap = true;          // IBLB_OVERLAP
    // deep slab cycles: the interior's edge waves wait on a device word the comm stream's boundary
    // sweeps signal (IBLB_EDGE_FLAG, default on) instead of the compute queue waiting for ev_bnd
    int edge_flag = 1;  // 1: two-way device handshake, 2: one way (interior waits only), 0: queue waits
    unsigned* sig = nullptr;      // device words: [0] sequence number of the last boundary launch done,
                                  // [16] edge waves of the slab interiors done (ctx_step.hip:deep_slab_step),
                                  // [24] band cycles whose exchange landed (ctx_band.hip:band_step)
    unsigned sig_n = 0;           // boundary launches signalled so far (the value of the last one)
    unsigned done_n = 0;          // interior edge waves launched so far (the done word's value once they end)
    unsigned bx_n = 0;            // band cycles whose exchange the level-0 IB signalled in sig[24] (ctx_band.hip)
    bool bx_dev = false;          // this band cycle's boundary sweeps wait on sig[24] (set by band_step)
    bool bnd_in_end = false;      // the last band cycle's band_end follows its boundary sweeps (ev_bnd)
    bool int_unrec = false;       // the last interior carried no event: ev_int is recorded on demand
    unsigned* sig_err = nullptr;  // host-coherent word: an edge wave's bounded wait timed out
    // the device waits' bound (IBLB_WAIT_TIMEOUT_S / iblb_set_wait_timeout, default 600 s): wall-clock
    // time, in ticks of the device's constant clock (hipDeviceAttributeWallClockRate)
    double wait_timeout_s = 600.;
    double clock_hz = 0.;  // the device wall clock's rate
    unsigned long long wait_ticks = 0;
    long long dev_wait_launches = 0;  // launches whose waves waited on a device word (iblb_timing)
    int deep_kinfo[4] = {0, 0, 0, 0};  // the last deep launch's build: MODE, VS, waves per SIMD, VGPRs (iblb_timing)
    // test hold (IBLB_TEST_HOLD=<n>:<ms>): exchange number n since the attach (0-based) starts after a
    // one-wave kernel that a host thread releases ms milliseconds after its submission, as if a
    // neighbour rank reached that exchange late (tests/test_gpu_wait.py)
    long long hold_x = -1, n_exch = 0;
    int hold_ms = 0;
    unsigned* hold_word = nullptr;  // host-coherent
    std::thread hold_thread;
    // profiling
    int prof = 0;  // 1: events around every launch; 2: the deep launches' own signals only (iblb_set_profiling)
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    double fused_ms = 0., ib_ms = 0., halo_ms = 0., sweep_ms = 0., sweepk_ms = 0.;
    long long fused_launches = 0, fused_cells = 0, sweep_launches = 0, sweep_cells = 0, sweepk_launches = 0,
              sweepk_cells = 0;
    long long band_cycles = 0, band_merged_cycles = 0, band_par_cycles = 0;  // IB band cycles run (counted without events too)
    long long deep_launches = 0, deep_iterations = 0;  // deep launches and the iterations they advanced (no events needed)
    bool band_own_build = false;  // the band cycle's deep sweep in the configured (not the chain-friendly) build
    struct EvRec { int kind; size_t idx; long long cells; };
    std::vector<EvRec> ev_kind;
    std::string err;
};

namespace iblbh {

int fail(iblb_ctx* c, int code, const std::string& msg);
int hip_fail(iblb_ctx* c, hipError_t e, const char* what);

#define HIP_TRY(c, expr)                                               \
    do {                                                               \
        hipError_t e_ = (expr);                                        \
        if (e_ != hipSuccess) return ::iblbh::hip_fail((c), e_, #expr); \
    } while (0)

#define NCCL_TRY(c, expr)                                                                                      \
    do {                                                                                                       \
        ncclResult_t r_ = (expr);                                                                              \
        if (r_ != ncclSuccess)                                                                                 \
            return ::iblbh::fail((c), IBLB_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_));       \
    } while (0)

template <typename T>
inline T* gptr(iblb_ctx* c, int which) { return (T*)c->g[which]; }

inline bool single_slab(const iblb_ctx* c) {
    return c->ncol == c->nx && c->transport != TR_LOCAL && c->nranks <= 1 && !c->self_ring;
}
inline bool rccl_multi(const iblb_ctx* c) { return c->transport == TR_RCCL && (c->nranks > 1 || c->self_ring); }
inline bool ib_active(const iblb_ctx* c) { return c->max_points > 0 && c->ns > 0; }
inline bool is_f64(const iblb_ctx* c) { return c->prec == IBLB_PREC_F64; }

// schedule entry of iteration it (clamped to the last one)
inline int sched_entry(const iblb_ctx* c, long long it) {
    const long long e = it - c->sch_t0;
    return (int)std::max(0LL, std::min(e, (long long)c->sch_n - 1));
}
template <typename P>
inline P* sched_ptr(P* base, const iblb_ctx* c, int e, int per_point) { return base + (size_t)e * per_point * c->ns; }
// the current points become those of schedule entry e (no copy: launches and readers take pts_*)
inline void sched_use(iblb_ctx* c, int e) {
    if (c->sch_n > 0) c->sch_cur = e;
}
// arrays of the current points: the schedule entry in use, else the static points
inline const float* pts_s(const iblb_ctx* c) {
    return c->sch_n > 0 && c->sch_cur >= 0 ? sched_ptr(c->d_sch_s, c, c->sch_cur, 2) : c->d_s;
}
inline const float* pts_us(const iblb_ctx* c) {
    return c->sch_n > 0 && c->sch_cur >= 0 ? sched_ptr(c->d_sch_us, c, c->sch_cur, 2) : c->d_us;
}
inline const int* pts_eps(const iblb_ctx* c) {
    return c->sch_n > 0 && c->sch_cur >= 0 ? sched_ptr(c->d_sch_eps, c, c->sch_cur, 1) : c->d_eps;
}
// the points of iteration it (a schedule entry, or the static points)
inline void pts_of(const iblb_ctx* c, long long it, const float** s, const float** us, const int** e) {
    if (c->sch_n > 0) {
        const int k = sched_entry(c, it);
        *s = sched_ptr(c->d_sch_s, c, k, 2);
        *us = sched_ptr(c->d_sch_us, c, k, 2);
        *e = sched_ptr(c->d_sch_eps, c, k, 1);
    } else {
        *s = c->d_s;
        *us = c->d_us;
        *e = c->d_eps;
    }
}

// periodic images of a lone slab: the edge columns of buffer g itself
template <typename T>
Halo<T> halo_at(const iblb_ctx* c, const T* g) {
    Halo<T> H;
    for (int p = 0; p < 3; ++p) {
        H.left[p] = g + left_plane(p) * c->L.plane + (long)(c->L.ncol - 1) * c->L.col;
        H.right[p] = g + right_plane(p) * c->L.plane;
    }
    return H;
}
// ghost columns -1 and ncol of buffer g
template <typename T>
Halo<T> ghost_halo(const iblb_ctx* c, const T* g) {
    Halo<T> H;
    for (int p = 0; p < 3; ++p) {
        H.left[p] = g + left_plane(p) * c->L.plane - c->L.col;
        H.right[p] = g + right_plane(p) * c->L.plane + (long)c->L.ncol * c->L.col;
    }
    return H;
}
template <typename T>
Halo<T> halo_of(iblb_ctx* c, int which) {
    const T* g = gptr<T>(c, which);
    return single_slab(c) ? halo_at<T>(c, g) : ghost_halo<T>(c, g);
}

// ---- profiling (iblb_ctx.hip) ----
int ev_begin(iblb_ctx* c, size_t* idx, hipStream_t st = nullptr);
int ev_end(iblb_ctx* c, size_t idx, int kind, long long cells = 0, hipStream_t st = nullptr);
// timing events that a launch carries itself (hipExtLaunchKernelGGL start / stop: the kernel's own
// dispatch and completion signals, no marker packets); null when not profiling
int ev_kernel(iblb_ctx* c, size_t* idx, hipEvent_t* start, hipEvent_t* stop);
int ev_kernel_end(iblb_ctx* c, size_t idx, int kind, long long cells);

// ---- halo / force (ctx_step.hip) ----
int rccl_order(iblb_ctx* c, hipStream_t st);
int join_comm(iblb_ctx* c);
int exchange(iblb_ctx* c, hipStream_t st, int d);
int fill_ghosts_periodic(iblb_ctx* c, int which, int d, hipStream_t st);
int ensure_halo(iblb_ctx* c);
int ensure_force(iblb_ctx* c);
int ib_ghost(iblb_ctx* c, const void* g, int gc, int clo, int chi, const float* s, const float* us, const int* eps,
             int part, hipStream_t st, unsigned* sig = nullptr, unsigned sig_val = 0, int wlo = 0, int whi = 0);
int check_ready(iblb_ctx* c);
int check_wait_err(iblb_ctx* c);  // after a synchronize: did an edge wave's wait time out?
int set_wait_ticks(iblb_ctx* c);  // wait_ticks from wait_timeout_s and the device's wall-clock rate
int hold_release(iblb_ctx* c);    // join the test hold's host thread (IBLB_TEST_HOLD)
int prepare_read(iblb_ctx* c);
int free_boot(iblb_ctx* c);
int alloc_zero(iblb_ctx* c, void** p, size_t bytes);
int run_cilia(iblb_ctx* c);
template <typename T>
Sweep2Args<T> sweep_args(iblb_ctx* c, int col_begin, int col_step, int col_end, int nsweep, int W);

// ---- band cycle (ctx_band.hip) ----
bool band_ready(const iblb_ctx* c);
int band_step_any(iblb_ctx* c);
int plan_bands(iblb_ctx* c, const std::vector<float>& xy);
int plan_cycle(iblb_ctx* c);
int band_join(iblb_ctx* c);     // the context's stream after a run of band cycles
int retire_points(iblb_ctx* c);  // owed force evaluated; an active schedule entry becomes the static points
int cilia_schedule(iblb_ctx* c, int n);  // cilia kinematics of the next n iterations as a schedule
int cilia_schedule_end(iblb_ctx* c);
bool band_possible(const iblb_ctx* c);  // the band cycle may run on this context (points aside)
int band_release(iblb_ctx* c);  // streams, events, pinned tables, scratch buffers

}  // namespace iblbh
