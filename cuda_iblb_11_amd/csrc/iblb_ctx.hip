// iblb_ctx.hip — the fused context API of include/iblb.h: state, time stepping, slab
// decomposition (local and RCCL transports), readers in the reference layouts.
//
// Time-step bookkeeping.  The reference iteration (main.cu:852-909) is
//   f0,F = equilibrium(u^t, rho^t, force^t); f1 = collision(f^t); f^{t+1} = stream(f1);
//   rho^{t+1}, u_raw = macro(f^{t+1}); F_s = interpolate(...); force^{t+1}, u^{t+1} = spread(...)
// The context stores g = f1^{t-1} (post-collision, not yet streamed).  One fused launch
// pulls f^t from g, recomputes rho^t and u^t = (sum c f + force^t/2)/rho^t, collides and
// stores f1^t.  force^t (the IB part of the PREVIOUS reference iteration) is computed
// lazily just before it is needed — before the next collide, before a reader, or before
// the Lagrangian points change — so every call sees exactly the reference's state.
// The flux term q(u^t) the reference adds at the end of iteration t-1 is added by the
// collide of step t; iblb_get_flux() adds the not-yet-collided last term on demand.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/iblb.h"

#include "cilia_kernels.h"
#include "iblb_kernels.h"

using namespace iblb;

extern "C" {
static int reset_cilia_state(iblb_ctx* c);
}

namespace {

enum Phase { PH_EMPTY = 0, PH_BOOT = 1, PH_RUN = 2 };
enum IbState { IB_NONE = 0, IB_PENDING = 1, IB_READY = 2 };
enum Transport { TR_NONE = 0, TR_LOCAL = 1, TR_RCCL = 2 };

constexpr long GUARD = 512;  // elements in front of / behind every population buffer

std::string g_create_error;

long env_long(const char* name, long dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::strtol(v, nullptr, 10) : dflt;
}

}  // namespace

struct iblb_ctx {
    iblb_config cfg{};
    int nx = 0, ny = 0, x_begin = 0, ncol = 0;
    int prec = IBLB_PREC_F64;
    size_t esize = 8;
    int V = 2, nch = 1;
    Layout L{};
    long fplane = 0;
    int device = 0;
    int variant = 0;  // collide-stream kernel variant (IBLB_FUSED_VARIANT, tuning only)
    // two iterations per launch (lbm_sweep.hip) where no IB force is owed in between:
    // IBLB_SWEEP (on), IBLB_SWEEP_W columns per wave, IBLB_SWEEP_VS cells per lane, variant
    bool sweep_on = true;
    int sweep_w = 4, sweep_vs = 2, sweep_variant = 1, sweep_map = 2, sweep_alt = 1;
    // K = 3 .. 6 iterations per launch on a lone slab (IBLB_SWEEP_DEPTH): columns per wave, cells per lane
    int sweep_depth = 2, deep_w = 4, deep_vs = 2, deep_variant = 1, deep_balance = 1, deep_bnd_vs = 2, deep_slab_vs = 1;
    int reserved_cus = 0, ncu = 0;  // CUs kept free of the compute stream (RCCL groups), device CUs
    std::vector<uint32_t> comp_mask;  // the compute stream's CU mask when reserved_cus > 0
    hipStream_t stream = nullptr;
    Coef coef{};
    KConst kc{};  // collide constants folded from coef (kernel arguments)
    // populations: two buffers in one allocation (deterministic relative placement of the
    // 18 streams the collide-stream kernel touches), `cur` holds the state
    char* g_alloc = nullptr;
    void* g[2] = {nullptr, nullptr};
    int cur = 0;
    // halo exchange buffers (multi-slab): 3 slots of `col` elements each, guarded
    char* halo_alloc = nullptr;
    void* recv_left = nullptr;
    void* recv_right = nullptr;
    void* send_left = nullptr;
    void* send_right = nullptr;
    // boot arrays (slab layout)
    double* rho0 = nullptr;
    double* u0 = nullptr;
    double* force0 = nullptr;
    // immersed boundary
    int max_points = 0, ns = 0;
    // on-device cilia kinematics (iblb_set_cilia)
    bool cilia_on = false;
    iblb_cilia cilia{};
    float* cil_samples = nullptr;  // the reference's d_boundary [5 * 9600 * c_num]
    float* cil_lasts = nullptr;    // [2 * 9600 * c_num]
    float* cil_bpoints = nullptr;  // [5 * 96 * c_num]
    float* d_s = nullptr;
    float* d_us = nullptr;
    float* d_Fs = nullptr;
    int* d_eps = nullptr;
    float* d_Fs_sum = nullptr;  // F_s summed over an RCCL group (reader scratch)
    // points given ahead (iblb_set_lagrangian_steps): entry i is used by iteration sch_t0 + i;
    // d_s / d_us / d_eps hold the entry of the current iteration (sch_cur)
    float* d_sch_s = nullptr;
    float* d_sch_us = nullptr;
    int* d_sch_eps = nullptr;
    size_t sch_cap = 0;  // entries allocated
    int sch_n = 0, sch_cur = -1;
    long long sch_t0 = 0;
    // band plans of a schedule: one per cycle from the x coordinates of the cycle's entries
    // (host copies), installed when the cycle's bands differ from the installed ones
    std::vector<float> sch_x;       // [sch_n][ns][2]: point coordinates (x, y) of the schedule
    std::vector<float> sch_x_prev;  // the points before the schedule (their force may be owed)
    std::vector<std::array<int, 4>> band_b;  // merged forced patches {x0, x1, y0, y1} of the installed plan
    // pinned host staging of the uploaded tables: a ring, each slot reused only after its copy
    int* band_pin[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t band_pin_cap = 0;  // ints per slot
    hipEvent_t band_pin_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    int band_pin_i = 0;
    bool band_sticky = false;                 // keep the reserved XCDs while a schedule runs
    double* fdense = nullptr;
    uint8_t* flags = nullptr;
    // IB bands of the K-iteration cycle (lone slab, points fixed between iblb_set_lagrangian
    // calls): the columns an owed force can reach within K iterations advance one iteration per
    // launch (trapezoid through sbuf), the force-free gaps between them in one deep sweep
    int band_on = 1;                     // IBLB_IB_BAND
    bool band_valid = false;
    int* d_band = nullptr;               // level column tables, then the deep sweep table
    size_t band_cap = 0;                 // ints allocated at d_band
    std::vector<int> band_off, band_n;   // level j = 0 .. K-1: offset / entries in d_band
    std::vector<int> band_nchl;          // level j: chunks per entry (patch rows) launched
    int band_sweep_off = 0, band_nsweep = 0;
    long long band_deep_lu = 0, band_lu = 0;  // cells of the deep sweep / of all trapezoid levels
    int band_flux = -1;                  // flux column if a band outputs it, else -1
    // the band chain as ONE launch (band_kernel: a workgroup per patch runs its whole trapezoid,
    // IB included; IBLB_BAND_FUSED=1) instead of 2K dependent launches (default: one workgroup
    // per patch is latency-bound, K3 0.25 vs 0.09 ms per cycle, profiles/r02ad)
    int band_fused = 0;
    // the cycle's deep sweep over every column (IBLB_BAND_FULL, default) instead of the table of
    // gaps and band columns outside the patch rows: the patch rows it gets wrong (no force) are
    // overwritten by the trapezoid's last level, which waits for it (ev_bd)
    int band_full = 1;
    // the launches read the plan's tables straight from its pinned slot (IBLB_BAND_HOSTTAB,
    // default): a new plan of moving points costs no copy on the cycle's critical path
    int band_hosttab = 1;
    int* band_tab = nullptr;   // the tables the cycle's launches read (d_band or a pinned slot)
    int band_pin_cur = -1;     // the pinned slot band_tab points into (its event: the cycle's end)
    int band_tail_ds = 1;  // IBLB_BAND_TAIL_DS
    hipEvent_t ev_bd = nullptr;
    int band_npatch = 0, band_pt_off = 0;  // patches; their table in d_band (BAND_PT ints each)
    char* s_alloc = nullptr;             // two scratch population buffers of the trapezoid
    void* sbuf[2] = {nullptr, nullptr};
    long buf_elems = 0, buf_gap = 0;
    // the band chain beside the deep sweep: CUs reserved for it (whole XCDs, IBLB_BAND_RESERVE_CUS;
    // 0 = both on the compute stream, in sequence)
    int band_reserve = 0;
    hipStream_t band_st = nullptr;   // the band chain (masked to the reserved CUs)
    hipStream_t deep_st = nullptr;   // the cycle's deep sweep (masked to the other CUs)
    hipEvent_t ev_b0 = nullptr, ev_b1 = nullptr, ev_b2 = nullptr;
    // flux: d_Q[0] cumulative, d_Q[1] scratch
    double* d_Q = nullptr;
    // state machine
    int phase = PH_EMPTY;
    long long t = 0;
    int ib_state = IB_NONE;
    bool halo_valid = false;
    bool halo_ib = false;  // the received halo carries the IB slots (IB_HALO_SLOTS)
    bool send_sweep = false;  // the send buffers hold the 2-step halo of the current state
    int send_deep = 0;        // ... or the deep halo of this depth (deep_slot layout), 0 = none
    int halo_slots = HALO_SLOTS;  // slots per halo buffer (IB_HALO_SLOTS when IB-capable)
    // transport
    int transport = TR_NONE;
    iblb_ctx* left = nullptr;
    iblb_ctx* right = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool self_ring = false;  // one rank that is its own neighbour over RCCL (IBLB_RCCL_SELF, rehearsal)
    std::vector<int> slab_begin, slab_count;  // every rank's columns (RCCL group)
    hipStream_t comm_stream = nullptr;  // RCCL halo exchange, overlapped with the interior
    hipEvent_t ev_bnd = nullptr;  // boundary columns + send buffers of the state written (either stream)
    hipEvent_t ev_int = nullptr;  // compute-stream work of the last step done
    bool deep_chain = false;      // the last compute work is a deep slab cycle's (interior first) ...
    long long deep_chain_t = -1;  // ... that ended at this t with this cur: ev_int follows its interior
    int deep_chain_cur = -1;
    hipEvent_t ev_pre = nullptr;  // compute-stream work before the interior sweep (sweep order 1)
    bool overlap = true;
    int sweep_order = 0;          // IBLB_SWEEP_ORDER: 1 = the host submits the interior sweep first
    int deep_order = 1;           // IBLB_DEEP_ORDER: the same for the deep slab cycle (default: 512 x 4096
                                  // self ring 0.0268 vs 0.0317 ms/iteration, profiles/r01l_*)
    // profiling
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    double fused_ms = 0., ib_ms = 0., halo_ms = 0., sweep_ms = 0., sweepk_ms = 0.;
    long long fused_launches = 0, fused_cells = 0, sweep_launches = 0, sweep_cells = 0, sweepk_launches = 0,
              sweepk_cells = 0;
    struct EvRec { int kind; size_t idx; long long cells; };
    std::vector<EvRec> ev_kind;
    std::string err;
};

namespace {

int fail(iblb_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    else g_create_error = msg;
    return code;
}

int hip_fail(iblb_ctx* c, hipError_t e, const char* what) {
    return fail(c, e == hipErrorOutOfMemory ? IBLB_ERR_NOMEM : IBLB_ERR_HIP,
                std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(c, expr)                                               \
    do {                                                               \
        hipError_t e_ = (expr);                                        \
        if (e_ != hipSuccess) return hip_fail((c), e_, #expr);         \
    } while (0)

#define NCCL_TRY(c, expr)                                                                           \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess) return fail((c), IBLB_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

template <typename T>
T* gptr(iblb_ctx* c, int which) { return (T*)c->g[which]; }

bool single_slab(const iblb_ctx* c) {
    return c->ncol == c->nx && c->transport != TR_LOCAL && c->nranks <= 1 && !c->self_ring;
}
bool rccl_multi(const iblb_ctx* c) { return c->transport == TR_RCCL && (c->nranks > 1 || c->self_ring); }
bool ib_active(const iblb_ctx* c) { return c->max_points > 0 && c->ns > 0; }

// schedule entry of iteration it (clamped to the last one)
int sched_entry(const iblb_ctx* c, long long it) {
    const long long e = it - c->sch_t0;
    return (int)std::max(0LL, std::min(e, (long long)c->sch_n - 1));
}
template <typename P>
P* sched_ptr(P* base, const iblb_ctx* c, int e, int per_point) { return base + (size_t)e * per_point * c->ns; }

// the current points become those of schedule entry e (no copy: the IB launches and readers
// take the entry's arrays, pts_*)
int sched_use(iblb_ctx* c, int e) {
    if (c->sch_n > 0) c->sch_cur = e;
    return IBLB_OK;
}
// arrays of the current points: the schedule entry in use, else the static points
const float* pts_s(const iblb_ctx* c) { return c->sch_n > 0 && c->sch_cur >= 0 ? sched_ptr(c->d_sch_s, c, c->sch_cur, 2) : c->d_s; }
const float* pts_us(const iblb_ctx* c) {
    return c->sch_n > 0 && c->sch_cur >= 0 ? sched_ptr(c->d_sch_us, c, c->sch_cur, 2) : c->d_us;
}
const int* pts_eps(const iblb_ctx* c) {
    return c->sch_n > 0 && c->sch_cur >= 0 ? sched_ptr(c->d_sch_eps, c, c->sch_cur, 1) : c->d_eps;
}

// periodic images of a lone slab: the edge columns of the buffer g itself
template <typename T>
Halo<T> halo_at(iblb_ctx* c, const T* g) {
    Halo<T> H;
    const Layout& L = c->L;
    for (int p = 0; p < 3; ++p) {
        H.left[p] = g + left_plane(p) * L.plane + (long)(L.ncol - 1) * L.col;
        H.right[p] = g + right_plane(p) * L.plane;
    }
    return H;
}

template <typename T>
Halo<T> halo_of(iblb_ctx* c, int which) {
    Halo<T> H;
    const Layout& L = c->L;
    if (single_slab(c)) {
        const T* g = gptr<T>(c, which);
        for (int p = 0; p < 3; ++p) {
            H.left[p] = g + left_plane(p) * L.plane + (long)(L.ncol - 1) * L.col;
            H.right[p] = g + right_plane(p) * L.plane;
        }
    } else {
        for (int p = 0; p < 3; ++p) {
            H.left[p] = (const T*)c->recv_left + p * L.rows;
            H.right[p] = (const T*)c->recv_right + p * L.rows;
        }
    }
    return H;
}

template <typename T>
void send_ptrs(iblb_ctx* c, T* sl[3], T* sr[3]) {
    for (int p = 0; p < 3; ++p) {
        sl[p] = single_slab(c) ? nullptr : (T*)c->send_left + p * c->L.rows;
        sr[p] = single_slab(c) ? nullptr : (T*)c->send_right + p * c->L.rows;
    }
}

// ---- profiling --------------------------------------------------------------------------
enum EvKind { EV_FUSED = 0, EV_IB = 1, EV_HALO = 2, EV_SWEEP = 3, EV_SWEEPK = 4 };

void ev_account(iblb_ctx* c, const iblb_ctx::EvRec& r, float ms) {
    if (r.kind == EV_FUSED) { c->fused_ms += ms; c->fused_launches++; c->fused_cells += r.cells; }
    else if (r.kind == EV_SWEEP) { c->sweep_ms += ms; c->sweep_launches++; c->sweep_cells += r.cells; }
    else if (r.kind == EV_SWEEPK) { c->sweepk_ms += ms; c->sweepk_launches++; c->sweepk_cells += r.cells; }
    else if (r.kind == EV_IB) c->ib_ms += ms;
    else c->halo_ms += ms;
}

int ev_begin(iblb_ctx* c, size_t* idx, hipStream_t st = nullptr) {
    if (!c->prof) return IBLB_OK;
    if (c->ev_used + 2 > c->ev_pool.size()) {
        // timing events bracket kernels of this device only: no system-scope fence
        // (IBLB_PROF_EVENT_FENCE=0 restores HIP's default release / acquire at system scope)
        const unsigned flags = env_long("IBLB_PROF_EVENT_FENCE", 1) ? hipEventDisableSystemFence : 0u;
        for (int k = 0; k < 64; ++k) {
            hipEvent_t e;
            HIP_TRY(c, hipEventCreateWithFlags(&e, flags));
            c->ev_pool.push_back(e);
        }
    }
    *idx = c->ev_used;
    c->ev_used += 2;
    HIP_TRY(c, hipEventRecord(c->ev_pool[*idx], st ? st : c->stream));
    return IBLB_OK;
}

int ev_end(iblb_ctx* c, size_t idx, int kind, long long cells = 0, hipStream_t st = nullptr) {
    if (!c->prof) return IBLB_OK;
    HIP_TRY(c, hipEventRecord(c->ev_pool[idx + 1], st ? st : c->stream));
    c->ev_kind.push_back({kind, idx, cells});
    if (c->ev_used >= 8192) {  // bound the pool: drain what is recorded
        HIP_TRY(c, hipEventSynchronize(c->ev_pool[idx + 1]));
        if (c->comm_stream) HIP_TRY(c, hipStreamSynchronize(c->comm_stream));
        if (c->band_st) HIP_TRY(c, hipStreamSynchronize(c->band_st));
        if (c->deep_st) HIP_TRY(c, hipStreamSynchronize(c->deep_st));
        for (auto& r : c->ev_kind) {
            float ms = 0.f;
            HIP_TRY(c, hipEventElapsedTime(&ms, c->ev_pool[r.idx], c->ev_pool[r.idx + 1]));
            ev_account(c, r, ms);
        }
        c->ev_kind.clear();
        c->ev_used = 0;
    }
    return IBLB_OK;
}

// ---- halo exchange ----------------------------------------------------------------------
// IB slots of the send buffers (slots 0-2 come from the collide)
template <typename T>
int pack_ib(iblb_ctx* c, hipStream_t st) {
    HIP_TRY(c, launch_pack_ib_halo<T>(gptr<T>(c, c->cur), c->L, (T*)c->send_left, (T*)c->send_right, st));
    return IBLB_OK;
}
int pack_ib_any(iblb_ctx* c, hipStream_t st) {
    if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
    return c->prec == IBLB_PREC_F64 ? pack_ib<double>(c, st) : pack_ib<float>(c, st);
}

// ib: also carry the IB slots (the owed force is evaluated from this halo); sweep: the 2-step
// halo (the send buffers hold it: written by the boundary sweep or packed)
int exchange_rccl(iblb_ctx* c, hipStream_t st, bool ib = false, bool sweep = false, int nslots = 0) {
    size_t ev = 0;
    int rc;
    if (ib && (rc = pack_ib_any(c, st))) return rc;
    if (ib) c->send_sweep = false;  // slots 3.. now carry the IB halo
    if (ib) c->send_deep = 0;
    if ((rc = ev_begin(c, &ev, st))) return rc;
    if (nslots <= 0) nslots = ib ? IB_HALO_SLOTS : (sweep ? SWEEP_HALO_SLOTS : HALO_SLOTS);
    const size_t n = (size_t)nslots * c->L.rows;
    const ncclDataType_t dt = c->prec == IBLB_PREC_F64 ? ncclFloat64 : ncclFloat32;
    const int lr = (c->rank + c->nranks - 1) % c->nranks, rr = (c->rank + 1) % c->nranks;
    NCCL_TRY(c, ncclGroupStart());
    NCCL_TRY(c, ncclSend(c->send_right, n, dt, rr, c->comm, st));
    NCCL_TRY(c, ncclSend(c->send_left, n, dt, lr, c->comm, st));
    NCCL_TRY(c, ncclRecv(c->recv_left, n, dt, lr, c->comm, st));
    NCCL_TRY(c, ncclRecv(c->recv_right, n, dt, rr, c->comm, st));
    NCCL_TRY(c, ncclGroupEnd());
    c->halo_valid = true;
    c->halo_ib = ib;
    return ev_end(c, ev, EV_HALO, 0, st);
}

// local group: the neighbours' send buffers are complete (group_exchange packed them)
int exchange_local(iblb_ctx* c, bool ib) {
    const size_t bytes = (size_t)(ib ? IB_HALO_SLOTS : HALO_SLOTS) * c->L.rows * c->esize;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(c->recv_left, c->left->send_right, bytes, hipMemcpyDefault, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->recv_right, c->right->send_left, bytes, hipMemcpyDefault, c->stream));
    c->halo_valid = true;
    c->halo_ib = ib;
    return IBLB_OK;
}

// send buffers of the state in g[cur] (normally written by the collide that produced it)
int pack_send(iblb_ctx* c) {
    if (c->phase != PH_RUN || single_slab(c) || c->transport == TR_NONE) return IBLB_OK;
    const size_t n = (size_t)c->ny * c->esize;
    char* g = (char*)c->g[c->cur];
    for (int p = 0; p < 3; ++p) {
        const char* r = g + ((size_t)left_plane(p) * c->L.plane + (size_t)(c->ncol - 1) * c->L.col) * c->esize;
        const char* l = g + (size_t)right_plane(p) * c->L.plane * c->esize;
        HIP_TRY(c, hipMemcpyAsync((char*)c->send_right + p * c->L.rows * c->esize, r, n, hipMemcpyDeviceToDevice,
                                  c->stream));
        HIP_TRY(c, hipMemcpyAsync((char*)c->send_left + p * c->L.rows * c->esize, l, n, hipMemcpyDeviceToDevice,
                                  c->stream));
    }
    c->send_sweep = false;
    c->send_deep = 0;
    if (rccl_multi(c)) {
        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
    }
    return IBLB_OK;
}

// ---- immersed boundary ------------------------------------------------------------------
// Single slab: the whole IB of a step in one launch.  The dense force and its flags are clean
// here: the collide that consumed the previous force cleared both.
template <typename T>
int ib_single(iblb_ctx* c) {
    HIP_TRY(c, launch_ib_point<T>(gptr<T>(c, c->cur), c->L, halo_of<T>(c, c->cur), c->nx, c->ns, pts_s(c), pts_us(c),
                                  pts_eps(c), c->d_Fs, c->fdense, c->fplane, c->flags, c->nch, 64 * c->V, c->stream));
    c->ib_state = IB_READY;
    return IBLB_OK;
}

// Slab of a group: the points spreading into it, from the IB halo (no collective).
template <typename T>
int ib_slab(iblb_ctx* c) {
    IbHalo<T> X{(const T*)c->recv_left, (const T*)c->recv_right};
    HIP_TRY(c, launch_ib_slab<T>(gptr<T>(c, c->cur), c->L, X, c->nx, c->x_begin, c->ns, pts_s(c), pts_us(c), pts_eps(c),
                                 c->d_Fs, c->fdense, c->fplane, c->flags, c->nch, 64 * c->V, c->stream));
    c->ib_state = IB_READY;
    return IBLB_OK;
}

int ib_slab_any(iblb_ctx* c) {
    if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
    return c->prec == IBLB_PREC_F64 ? ib_slab<double>(c) : ib_slab<float>(c);
}

// halo of the current state for a context that is alone or in an RCCL group (local groups:
// group code); with an owed IB force it must carry the IB slots
int ensure_halo(iblb_ctx* c) {
    if (single_slab(c)) return IBLB_OK;
    const bool ib = c->ib_state == IB_PENDING;
    if (c->halo_valid && (c->halo_ib || !ib)) return IBLB_OK;
    if (c->transport == TR_RCCL) return exchange_rccl(c, c->stream, ib);
    return fail(c, IBLB_ERR_STATE, "slab halo not available: link the slabs (iblb_link_local / iblb_attach_rccl)");
}

int ensure_force(iblb_ctx* c) {
    if (c->ib_state != IB_PENDING) return IBLB_OK;
    if (c->transport == TR_LOCAL)
        return fail(c, IBLB_ERR_STATE, "local group: advance with iblb_group_step");
    int rc = ensure_halo(c);
    if (rc) return rc;
    size_t ev = 0;
    if ((rc = ev_begin(c, &ev))) return rc;
    if (single_slab(c)) {
        if ((rc = c->prec == IBLB_PREC_F64 ? ib_single<double>(c) : ib_single<float>(c))) return rc;
    } else {
        if ((rc = ib_slab_any(c))) return rc;
    }
    return ev_end(c, ev, EV_IB);
}

// ---- the step -----------------------------------------------------------------------------
template <typename T>
int launch_boot_step(iblb_ctx* c) {
    T* sl[3];
    T* sr[3];
    send_ptrs<T>(c, sl, sr);
    HIP_TRY(c, launch_boot<T>(gptr<T>(c, c->cur), gptr<T>(c, 1 - c->cur), c->L, c->rho0, c->u0, c->force0, c->fplane,
                              sl, sr, c->coef, c->kc, c->stream));
    return IBLB_OK;
}

template <typename T>
int launch_fused_step(iblb_ctx* c, int col_begin, int ncols, int col_step = 1, bool timed = true,
                      hipStream_t st = nullptr) {
    FusedArgs<T> a;
    a.src = gptr<T>(c, c->cur);
    a.dst = gptr<T>(c, 1 - c->cur);
    a.L = c->L;
    a.H = halo_of<T>(c, c->cur);
    send_ptrs<T>(c, a.send_left, a.send_right);
    a.col_begin = col_begin;
    a.col_step = col_step;
    a.ncols = ncols;
    a.cols = nullptr;
    a.nch = c->nch;
    const bool ib = c->ib_state == IB_READY;
    a.flags = ib ? c->flags : nullptr;
    a.fdense = c->fdense;
    a.fplane = c->fplane;
    const int fc = c->cfg.flux_column - c->x_begin;
    a.flux_col = (fc >= 0 && fc < c->ncol) ? fc : -1;
    a.flux_norm = c->cfg.flux_norm;
    a.Q = c->d_Q;
    a.c = c->coef;
    a.k = c->kc;
    a.variant = c->variant;
    size_t ev = 0;
    int rc = timed ? ev_begin(c, &ev) : IBLB_OK;
    if (rc) return rc;
    HIP_TRY(c, launch_fused<T>(a, st ? st : c->stream));
    return timed ? ev_end(c, ev, EV_FUSED, (long long)ncols * c->ny) : IBLB_OK;
}

int free_boot(iblb_ctx* c) {
    if (c->rho0) (void)hipFree(c->rho0);
    if (c->u0) (void)hipFree(c->u0);
    if (c->force0) (void)hipFree(c->force0);
    c->rho0 = c->u0 = c->force0 = nullptr;
    return IBLB_OK;
}

void after_step(iblb_ctx* c) {
    c->send_sweep = false;  // a one-step collide writes the one-step slots only
    c->send_deep = 0;
    c->cur = 1 - c->cur;
    c->t++;
    c->halo_valid = false;
    c->ib_state = ib_active(c) ? IB_PENDING : IB_NONE;
}

// RCCL slab, no IB force owed.  Step t on two streams:
//   comm:    exchange(t) [send buffers of g^{t-1}] -> wait int(t-1) -> boundary columns(t) -> ev_bnd
//   compute: (waited for ev_bnd = boundary(t-1) in step_one) -> interior columns(t) -> ev_int
// The interior needs nothing from the exchange, so the halo and the two boundary columns run
// beside it (on the CUs the collide leaves free, IBLB_RESERVE_CUS): the step costs the interior
// launch as long as exchange + boundary are shorter.  boundary(t) waits for interior(t-1): it
// reads columns 1 and ncol-2 of g^{t-1} and overwrites columns of the buffer interior(t-1) read.
template <typename T>
int overlapped_step(iblb_ctx* c) {
    int rc = exchange_rccl(c, c->comm_stream);
    if (rc) return rc;
    HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_int, 0));
    if ((rc = launch_fused_step<T>(c, 0, 2, c->ncol - 1, false, c->comm_stream))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_bnd, c->comm_stream));
    if ((rc = launch_fused_step<T>(c, 1, c->ncol - 2))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
    after_step(c);
    return IBLB_OK;
}

// RCCL slab with an IB force owed (force^t of the points of iteration t-1), step t on two streams:
//   compute: (join_comm: boundary(t-1)) -> IB of the inner points -> ev_pre -> interior columns
//            [3, ncol-3)(t) -> ev_int
//   comm:    wait int(t-1) -> IB halo pack + exchange(t) -> IB of the edge points -> wait ev_pre ->
//            boundary columns [0, 3) and [ncol-3, ncol)(t) -> ev_bnd
// Inner points (x_begin+2 <= x0 <= x_begin+ncol-3: nodes and pulls inside the slab) need no halo
// and spread into columns [1, ncol-2]; edge points need the IB halo and spread into columns
// <= 2 and >= ncol-3 only, so the interior collide waits for neither the exchange nor the edge
// IB.  boundary(t) waits for the inner IB (its columns 1, 2 / ncol-3, ncol-2 may hold inner
// forces) and for interior(t-1) (which read the columns it overwrites); interior(t) and the
// inner IB of t read columns boundary(t-1) wrote (join_comm).  next: the schedule entry the
// iteration's points switch to after the owed force is evaluated (-1: unchanged).
template <typename T>
int ib_overlapped_step(iblb_ctx* c, int next) {
    hipStream_t bs = c->comm_stream;
    IbHalo<T> X{(const T*)c->recv_left, (const T*)c->recv_right};
    int rc;
    HIP_TRY(c, launch_ib_slab<T>(gptr<T>(c, c->cur), c->L, X, c->nx, c->x_begin, c->ns, pts_s(c), pts_us(c), pts_eps(c),
                                 c->d_Fs, c->fdense, c->fplane, c->flags, c->nch, 64 * c->V, c->stream, 1));
    HIP_TRY(c, hipEventRecord(c->ev_pre, c->stream));
    HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_int, 0));
    if ((rc = exchange_rccl(c, bs, true))) return rc;
    HIP_TRY(c, launch_ib_slab<T>(gptr<T>(c, c->cur), c->L, X, c->nx, c->x_begin, c->ns, pts_s(c), pts_us(c), pts_eps(c),
                                 c->d_Fs, c->fdense, c->fplane, c->flags, c->nch, 64 * c->V, bs, 2));
    c->ib_state = IB_READY;
    if (next >= 0 && (rc = sched_use(c, next))) return rc;
    HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_pre, 0));
    if ((rc = launch_fused_step<T>(c, 0, 3, 1, false, bs))) return rc;
    if ((rc = launch_fused_step<T>(c, c->ncol - 3, 3, 1, false, bs))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
    if ((rc = launch_fused_step<T>(c, 3, c->ncol - 6))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
    after_step(c);
    return IBLB_OK;
}

// Compute stream after the boundary columns of the current state (they may have been written
// on the comm stream by an overlapped step).
int join_comm(iblb_ctx* c) {
    if (c->comm_stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_bnd, 0));
    return IBLB_OK;
}

// ---- two iterations per launch ---------------------------------------------------------------
// No IB force owed before or between the two iterations (no IB points, no cilia).  A lone slab:
// one launch.  A slab of an RCCL group (>= 4 columns): the 2-step halo exchange and the boundary
// sweeps (columns 0, 1, ncol-2, ncol-1) on the comm stream beside the interior sweep, like
// overlapped_step:
//   comm:    exchange(t) -> wait int(t-2) -> boundary(t) [+ 2-step send halo of g^{t+2}] -> ev_bnd
//   compute: (join_comm: boundary(t-2)) -> interior columns [2, ncol-2)(t) -> ev_int
bool sweep_ready(const iblb_ctx* c) {
    if (!c->sweep_on || c->phase != PH_RUN || c->cilia_on || ib_active(c) || c->ib_state != IB_NONE) return false;
    if (single_slab(c)) return c->ncol >= 2;
    return rccl_multi(c) && c->ncol >= 4;
}

template <typename T>
Sweep2Args<T> sweep_args(iblb_ctx* c, int col_begin, int col_step, int col_end, int nsweep, int W) {
    Sweep2Args<T> a{};
    a.src = gptr<T>(c, c->cur);
    a.dst = gptr<T>(c, 1 - c->cur);
    a.L = c->L;
    a.recv_left = (const T*)c->recv_left;
    a.recv_right = (const T*)c->recv_right;
    a.send_left = (T*)c->send_left;
    a.send_right = (T*)c->send_right;
    a.col_begin = col_begin;
    a.col_step = col_step;
    a.col_end = col_end;
    a.nsweep = nsweep;
    a.W = W;
    a.vs = c->sweep_vs;
    a.variant = c->sweep_variant;
    a.map = c->sweep_map;
    a.alt = c->sweep_alt;
    const int fc = c->cfg.flux_column - c->x_begin;
    a.flux_col = (fc >= 0 && fc < c->ncol) ? fc : -1;
    a.flux_norm = c->cfg.flux_norm;
    a.Q = c->d_Q;
    a.c = c->coef;
    a.k = c->kc;
    return a;
}

template <typename T>
int sweep_launch(iblb_ctx* c, const Sweep2Args<T>& a, bool slab, hipStream_t st, bool timed, long long cells) {
    size_t ev = 0;
    int rc = timed ? ev_begin(c, &ev, st) : IBLB_OK;
    if (rc) return rc;
    HIP_TRY(c, launch_sweep2<T>(a, slab, st));
    return timed ? ev_end(c, ev, EV_SWEEP, cells, st) : IBLB_OK;
}

void after_sweep(iblb_ctx* c) {
    c->cur = 1 - c->cur;
    c->t += 2;
    c->halo_valid = false;
}

// K = sweep_depth iterations per cycle on a slab of an RCCL group (ncol >= 2K): the deep halo
// (deep_slots(K) column-planes per side) exchanged and the boundary sweeps (output columns
// [0, K) and [ncol-K, ncol), which then pack the deep halo of the new state) on the comm stream
// beside the interior sweep [K, ncol-K), as sweep_step does for two iterations:
//   comm:    exchange(t) -> wait int(t-K) -> boundary(t) [+ deep halo of g^{t+K}] -> ev_bnd
//   compute: (join_comm: boundary(t-K)) -> interior(t) -> ev_int
template <typename T>
int deep_slab_step(iblb_ctx* c) {
    const int K = c->sweep_depth;
    const int W = std::max(1, c->deep_w);
    const bool ov = c->overlap;
    int rc = join_comm(c);
    if (rc) return rc;
    if (c->send_deep != K) {  // the send buffers hold another halo: pack the deep one now
        HIP_TRY(c, launch_pack_deep_halo<T>(gptr<T>(c, c->cur), c->L, K, (T*)c->send_left, (T*)c->send_right,
                                            c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
    }
    hipStream_t bs = ov ? c->comm_stream : c->stream;
    const int ni = c->ncol - 2 * K;  // interior [K, ncol-K): needs nothing from the halo
    auto interior = [&]() -> int {
        if (ni <= 0) return IBLB_OK;
        Sweep2Args<T> a = sweep_args<T>(c, K, c->deep_balance ? 0 : W, c->ncol - K, (ni + W - 1) / W, W);
        a.vs = c->deep_slab_vs;
        a.cus = c->ncu - c->reserved_cus;  // the compute stream's CU mask
        // the workgroups still go round-robin to all eight XCDs (mask bit i is a CU of XCD i % 8,
        // profiles/r02n_xcc_probe.txt), so the XCD-contiguous deal stays over eight
        a.xcds = (int)env_long("IBLB_DEEP_XCDS", 0);
        a.variant = c->deep_variant;
        if (a.map == 0) a.map = 2;
        size_t ev = 0;
        int r = ev_begin(c, &ev, c->stream);
        if (r) return r;
        HIP_TRY(c, launch_sweepk<T>(a, K, false, c->stream));
        return ev_end(c, ev, EV_SWEEPK, (long long)ni * c->ny, c->stream);
    };
    auto boundary = [&]() -> int {
        Sweep2Args<T> b = sweep_args<T>(c, 0, c->ncol - K, c->ncol, 2, K);  // [0, K) and [ncol-K, ncol)
        b.vs = c->deep_bnd_vs;
        b.variant = c->deep_variant;
        if (b.map == 0) b.map = 2;
        // the sweep also writes the next deep halo into the send buffers (no pack kernel)
        HIP_TRY(c, launch_sweepk<T>(b, K, true, bs));
        return IBLB_OK;
    };
    bool chain = false;
    if (ov && c->deep_order == 1) {
        // interior first: the launch the cycle time depends on leaves the host before the RCCL
        // group and the boundary launches.  The boundary waits for ev_int = the compute work
        // before this interior (interior(t-K), which read the columns it overwrites and wrote the
        // ones it reads).  Cycles back to back: the previous cycle recorded ev_int right after
        // interior(t-K), and ev_int is recorded again only after this cycle's boundary has taken
        // its wait, so the compute stream carries one wait and one record per cycle (each
        // cross-queue packet idles the compute queue for microseconds: 512 x 4096 self ring,
        // profiles/r02q_*: ~14 us per cycle between two interior sweeps with four of them, ~3 us
        // between back-to-back sweeps of a lone slab).
        if (!(c->deep_chain && c->deep_chain_t == c->t && c->deep_chain_cur == c->cur))
            HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        if ((rc = interior())) return rc;
        if ((rc = exchange_rccl(c, bs, false, false, deep_slots(K)))) return rc;
        HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_int, 0));
        if ((rc = boundary())) return rc;
        HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        chain = true;
    } else {
        if (!ov) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_bnd, 0));
        if ((rc = exchange_rccl(c, bs, false, false, deep_slots(K)))) return rc;
        if (ov) HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_int, 0));
        if ((rc = boundary())) return rc;
        if (ov) HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
        if ((rc = interior())) return rc;
        if (ov) HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        else {
            HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
            HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
            HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
        }
    }
    c->cur = 1 - c->cur;
    c->t += K;
    c->halo_valid = false;
    c->send_sweep = false;
    c->send_deep = K;
    c->deep_chain = chain;
    c->deep_chain_t = c->t;
    c->deep_chain_cur = c->cur;
    return IBLB_OK;
}

// K = sweep_depth iterations in one launch on a lone slab
template <typename T>
int sweepk_step(iblb_ctx* c) {
    const int W = std::max(1, c->deep_w);
    // balanced sweep widths (col_step 0: the launcher sizes the sweeps to whole rounds of waves)
    Sweep2Args<T> a = sweep_args<T>(c, 0, c->deep_balance ? 0 : W, c->ncol, (c->ncol + W - 1) / W, W);
    a.vs = c->deep_vs;
    a.variant = c->deep_variant;
    if (a.map == 0) a.map = 2;
    size_t ev = 0;
    int rc = ev_begin(c, &ev, c->stream);
    if (rc) return rc;
    HIP_TRY(c, launch_sweepk<T>(a, c->sweep_depth, false, c->stream));
    if ((rc = ev_end(c, ev, EV_SWEEPK, (long long)c->ncol * c->ny, c->stream))) return rc;
    c->cur = 1 - c->cur;
    c->t += c->sweep_depth;
    c->halo_valid = false;
    return IBLB_OK;
}

// ---- IB bands: K iterations per cycle with an owed force every iteration ---------------------
// Lone slab, points fixed (iblb_set_lagrangian; not cilia).  The force of iteration t+j is
// nonzero only in the forced columns F = [x0-1, x0+1] of the points, and the state of a column
// x after K iterations depends on forces within K-1 columns of x.  So the output columns within
// K-1 of F (the band) advance one iteration per launch over a shrinking trapezoid of columns
// (level j = 0 .. K-1 covers the band +- (K-1-j) columns, from g^t through the scratch buffers,
// the IB kernel evaluating force^{t+j} from level j-1 before it), and every other column in one
// deep sweep g^t -> g^{t+K} (sweep table over the gaps).  Both read g^t and write disjoint
// columns of g^{t+K}; each column is collided by the same kernels as one-step iterations, so the
// result equals K one-step iterations (the deep sweep is bit-identical to them, the trapezoid
// runs the one-step kernels themselves).
// the band cycle's geometry: a lone slab, or a slab of an RCCL group whose bands stay in its
// interior (the boundary columns then advance force-free from the deep halo, as deep_slab_step)
bool band_slab_ok(const iblb_ctx* c) {
    return rccl_multi(c) && c->overlap && c->comm_stream && c->ncol >= 4 * c->sweep_depth;
}
bool band_ready(const iblb_ctx* c) {
    return c->band_on && c->band_valid && (single_slab(c) || band_slab_ok(c)) && c->phase == PH_RUN &&
           !c->cilia_on && ib_active(c) && c->sweep_on && c->sweep_depth >= 3;
}

bool band_full_deep(const iblb_ctx* c);
template <typename T>
int band_deep(iblb_ctx* c, int K, hipStream_t ds);
template <typename T>
int band_chain(iblb_ctx* c, int K, const T* A, T* B, T* const S[2], bool slab, hipStream_t bs, hipStream_t ds);

template <typename T>
int band_step(iblb_ctx* c) {
    const int K = c->sweep_depth;
    int rc;
    const T* A = gptr<T>(c, c->cur);
    T* B = gptr<T>(c, 1 - c->cur);
    T* S[2] = {(T*)c->sbuf[0], (T*)c->sbuf[1]};
    // overlapped: the deep sweep on deep_st (masked to the CUs outside the reserved XCDs), the
    // band chain on band_st (the reserved XCDs).  The context's own stream keeps the whole chip
    // (iblb_get_stream hands it out; every other step runs on it): the two masked streams start
    // after its work so far, and it waits for both at the end of the cycle.
    //
    // A slab of an RCCL group (bands in its interior, every point's trapezoid inside its slab):
    // the compute stream runs the IB, the gaps' deep sweep and the band chain on interior columns
    // (none reads the halo); the comm stream exchanges the deep halo and advances the force-free
    // boundary columns [0, K), [ncol-K, ncol) exactly as deep_slab_step does.
    const bool slab = !single_slab(c);
    const bool ov = c->band_st != nullptr;
    hipStream_t bs = ov ? c->band_st : c->stream, ds = ov ? c->deep_st : c->stream;
    if (slab) {
        if ((rc = join_comm(c))) return rc;  // boundary(t-K) wrote columns the interior reads
        if (c->send_deep != K) {            // the send buffers hold another halo: pack the deep one
            HIP_TRY(c, launch_pack_deep_halo<T>(A, c->L, K, (T*)c->send_left, (T*)c->send_right, c->stream));
            HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
            HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
            HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
        }
        HIP_TRY(c, hipEventRecord(c->ev_pre, c->stream));
    }
    if (ov) {
        HIP_TRY(c, hipEventRecord(c->ev_b0, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_b0, 0));
        HIP_TRY(c, hipStreamWaitEvent(ds, c->ev_b0, 0));
    }
    if (c->band_fused) {
        // the deep sweep over the gaps, beside ONE band-kernel launch for every patch's trapezoid
        if ((rc = band_deep<T>(c, K, ds))) return rc;
        BandArgs<T> ba{};
        FusedArgs<T>& a = ba.f;
        a.L = c->L;
        for (int p = 0; p < 3; ++p) a.send_left[p] = a.send_right[p] = nullptr;
        a.cols = c->band_tab;
        a.nch = c->nch;
        a.row_tab = 1;
        a.flags = c->flags;
        a.fdense = c->fdense;
        a.fplane = c->fplane;
        a.flux_col = c->band_flux;  // ghost columns of the trapezoid never add flux
        a.flux_norm = c->cfg.flux_norm;
        a.Q = c->d_Q;
        a.c = c->coef;
        a.k = c->kc;
        a.variant = c->variant;
        for (int j = 0; j < K; ++j) {
            ba.src[j] = j == 0 ? A : S[(j - 1) & 1];
            ba.dst[j] = j == K - 1 ? B : S[j & 1];
            // level j's points: those of iteration t+j-1 (j = 0: the current ones, whose force is owed)
            ba.ps[j] = j == 0 ? pts_s(c) : c->d_s;
            ba.pus[j] = j == 0 ? pts_us(c) : c->d_us;
            ba.pe[j] = j == 0 ? pts_eps(c) : c->d_eps;
            if (j > 0 && c->sch_n > 0) {
                const int e = sched_entry(c, c->t + j - 1);
                ba.ps[j] = sched_ptr(c->d_sch_s, c, e, 2);
                ba.pus[j] = sched_ptr(c->d_sch_us, c, e, 2);
                ba.pe[j] = sched_ptr(c->d_sch_eps, c, e, 1);
            }
        }
        ba.H0 = halo_at<T>(c, A);
        ba.pt = c->band_tab + c->band_pt_off;
        ba.npatch = c->band_npatch;
        ba.K = K;
        ba.ib0 = c->ib_state == IB_PENDING;
        ba.ns = c->ns;
        ba.nx = c->nx;
        ba.x_begin = c->x_begin;
        ba.slab = slab;
        ba.X = IbHalo<T>{(const T*)c->recv_left, (const T*)c->recv_right};
        ba.F_s = c->d_Fs;
        ba.rows_per_chunk = 64 * c->V;
        size_t ev = 0;
        if ((rc = ev_begin(c, &ev, bs))) return rc;
        HIP_TRY(c, launch_band<T>(ba, bs));
        if ((rc = ev_end(c, ev, EV_FUSED, c->band_lu, bs))) return rc;
        c->ib_state = IB_READY;
    } else if ((rc = band_chain<T>(c, K, A, B, S, slab, bs, ds))) {
        return rc;
    }
    if (ov) {
        HIP_TRY(c, hipEventRecord(c->ev_b1, ds));
        HIP_TRY(c, hipEventRecord(c->ev_b2, bs));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_b1, 0));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_b2, 0));
    }
    if (slab) {
        // comm: deep halo exchange(t) -> (after the compute work before this cycle, which read
        // the columns the boundary sweeps overwrite) boundary sweeps -> deep halo of g^{t+K}
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        hipStream_t cs = c->comm_stream;
        if ((rc = exchange_rccl(c, cs, false, false, deep_slots(K)))) return rc;
        HIP_TRY(c, hipStreamWaitEvent(cs, c->ev_pre, 0));
        Sweep2Args<T> b = sweep_args<T>(c, 0, c->ncol - K, c->ncol, 2, K);  // [0, K) and [ncol-K, ncol)
        b.vs = c->deep_bnd_vs;
        b.variant = c->deep_variant;
        if (b.map == 0) b.map = 2;
        HIP_TRY(c, launch_sweepk<T>(b, K, true, cs));  // also packs the deep halo of B
        HIP_TRY(c, hipEventRecord(c->ev_bnd, cs));
        c->send_sweep = false;
        c->send_deep = K;
    }
    // the pinned table slot may be reused once every launch of this cycle has read it
    if (c->band_pin_cur >= 0) HIP_TRY(c, hipEventRecord(c->band_pin_ev[c->band_pin_cur], c->stream));
    c->cur = 1 - c->cur;
    c->t += K;
    c->halo_valid = false;
    c->ib_state = IB_PENDING;
    // the force now owed is that of iteration t+K-1's points
    return c->sch_n > 0 ? sched_use(c, sched_entry(c, c->t - 1)) : IBLB_OK;
}

// the deep sweep of a band cycle over the force-free gaps (and the band columns outside the
// patch rows): the sweep table of the plan
// the full-lattice deep sweep of a band cycle (band_full): every column of a lone slab, the
// interior [K, ncol-K) of a group slab; flux column in a band output: the table (the full sweep
// would add the patch rows' force-free flux)
bool band_full_deep(const iblb_ctx* c) { return c->band_full && !c->band_fused && c->band_flux < 0; }

template <typename T>
int band_deep(iblb_ctx* c, int K, hipStream_t ds) {
    if (band_full_deep(c)) {
        const bool slab = !single_slab(c);
        const int lo = slab ? K : 0, hi = slab ? c->ncol - K : c->ncol, n = hi - lo;
        if (n <= 0) return IBLB_OK;
        const int W = std::max(1, c->deep_w);
        Sweep2Args<T> d = sweep_args<T>(c, lo, c->deep_balance ? 0 : W, hi, (n + W - 1) / W, W);
        d.vs = c->deep_vs;
        d.variant = c->deep_variant;
        if (d.map == 0) d.map = 2;
        d.cus = (slab ? c->ncu - c->reserved_cus : c->ncu) - c->band_reserve;  // the deep stream's CUs
        if (!c->ncu) d.cus = 0;
        d.xcds = (int)env_long("IBLB_DEEP_XCDS", 0);
        size_t ev = 0;
        int rc = ev_begin(c, &ev, ds);
        if (rc) return rc;
        HIP_TRY(c, launch_sweepk<T>(d, K, false, ds));
        if ((rc = ev_end(c, ev, EV_SWEEPK, (long long)n * c->ny, ds))) return rc;
        if (c->band_st && !c->band_tail_ds) HIP_TRY(c, hipEventRecord(c->ev_bd, ds));
        return IBLB_OK;
    }
    if (c->band_nsweep <= 0) return IBLB_OK;
    Sweep2Args<T> d = sweep_args<T>(c, 0, 1, c->ncol, c->band_nsweep, std::max(1, c->deep_w));
    d.sweep_tab = c->band_tab + c->band_sweep_off;
    d.tab_rows = 1;
    d.vs = c->deep_vs;
    d.variant = c->deep_variant;
    if (d.map == 0) d.map = 2;
    d.xcds = (int)env_long("IBLB_DEEP_XCDS", 0);  // eight: masks take CUs of every XCD (interior above)
    size_t ev = 0;
    int rc = ev_begin(c, &ev, ds);
    if (rc) return rc;
    HIP_TRY(c, launch_sweepk<T>(d, K, false, ds));
    return ev_end(c, ev, EV_SWEEPK, c->band_deep_lu, ds);
}

// The band chain as 2K dependent launches (IBLB_BAND_FUSED=0): the IB of each level over every
// point, then the level's one-step launch over the trapezoid's entries.
template <typename T>
int band_chain(iblb_ctx* c, int K, const T* A, T* B, T* const S[2], bool slab, hipStream_t bs, hipStream_t ds) {
    int rc;
    // IB of one level: a lone slab with every point; a group slab with the points spreading into
    // it (all inner: no halo is read) and zero F_s for the others
    IbHalo<T> X{(const T*)c->recv_left, (const T*)c->recv_right};
    auto ib = [&](const T* g, const float* ps, const float* pus, const int* pe, hipStream_t st) -> hipError_t {
        if (!slab)
            return launch_ib_point<T>(g, c->L, halo_at<T>(c, g), c->nx, c->ns, ps, pus, pe, c->d_Fs, c->fdense, c->fplane,
                                      c->flags, c->nch, 64 * c->V, st);
        return launch_ib_slab<T>(g, c->L, X, c->nx, c->x_begin, c->ns, ps, pus, pe, c->d_Fs, c->fdense, c->fplane,
                                 c->flags, c->nch, 64 * c->V, st, 0);
    };
    if (c->ib_state == IB_PENDING) {  // force^t from g^t
        size_t ev = 0;
        if ((rc = ev_begin(c, &ev, bs))) return rc;
        HIP_TRY(c, ib(A, pts_s(c), pts_us(c), pts_eps(c), bs));
        if ((rc = ev_end(c, ev, EV_IB, 0, bs))) return rc;
        c->ib_state = IB_READY;
    }
    // deep sweep over the force-free gaps first: the chip is full while it runs
    if ((rc = band_deep<T>(c, K, ds))) return rc;
    for (int j = 0; j < K; ++j) {
        const T* src = j == 0 ? A : S[(j - 1) & 1];
        T* dst = j == K - 1 ? B : S[j & 1];
        if (j > 0) {  // force^{t+j} from the level below (valid on the band +- (K-j) columns)
            // with the points of iteration t+j-1 (a schedule given ahead, or the static points)
            const float *ps = c->d_s, *pus = c->d_us;
            const int* pe = c->d_eps;
            if (c->sch_n > 0) {
                const int e = sched_entry(c, c->t + j - 1);
                ps = sched_ptr(c->d_sch_s, c, e, 2);
                pus = sched_ptr(c->d_sch_us, c, e, 2);
                pe = sched_ptr(c->d_sch_eps, c, e, 1);
            }
            size_t ev = 0;
            if ((rc = ev_begin(c, &ev, bs))) return rc;
            HIP_TRY(c, ib(src, ps, pus, pe, bs));
            if ((rc = ev_end(c, ev, EV_IB, 0, bs))) return rc;
        }
        FusedArgs<T> a;
        a.src = src;
        a.dst = dst;
        a.L = c->L;
        a.H = halo_at<T>(c, src);
        for (int p = 0; p < 3; ++p) a.send_left[p] = a.send_right[p] = nullptr;
        a.cols = c->band_tab;
        a.col_begin = c->band_off[j];
        a.col_step = 1;
        a.ncols = c->band_n[j];
        a.nch = c->nch;
        a.row_tab = 1;
        a.nchl = c->band_nchl[j];
        a.store_rows = j == K - 1;  // the last level writes g^{t+K}: patch rows only
        a.flags = c->flags;
        a.fdense = c->fdense;
        a.fplane = c->fplane;
        a.flux_col = c->band_flux;  // ghost columns of the trapezoid never add flux
        a.flux_norm = c->cfg.flux_norm;
        a.Q = c->d_Q;
        a.c = c->coef;
        a.k = c->kc;
        a.variant = c->variant;
        // full deep sweep: it wrote (force-free) values into the patch rows of g^{t+K} too; the
        // last level overwrites them after it
        // (IBLB_BAND_TAIL_DS, default: the last level runs on the deep sweep's stream right behind
        // it, once the chain's IB of that level is done: one cross-stream hop less on the cycle's
        // critical path, and the deep stream's CUs)
        hipStream_t ls = bs;
        if (j == K - 1 && band_full_deep(c) && bs != ds) {
            if (c->band_tail_ds) {
                HIP_TRY(c, hipEventRecord(c->ev_bd, bs));
                HIP_TRY(c, hipStreamWaitEvent(ds, c->ev_bd, 0));
                ls = ds;
            } else {
                HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_bd, 0));
            }
        }
        size_t ev = 0;
        if ((rc = ev_begin(c, &ev, ls))) return rc;
        HIP_TRY(c, launch_fused<T>(a, ls));
        if ((rc = ev_end(c, ev, EV_FUSED, (long long)a.ncols * a.nchl * 64 * c->V, ls))) return rc;
    }
    return IBLB_OK;
}

template <typename T>
int sweep_step(iblb_ctx* c) {
    const int W = std::max(1, c->sweep_w);
    if (single_slab(c)) {
        int rc = sweep_launch<T>(c, sweep_args<T>(c, 0, W, c->ncol, (c->ncol + W - 1) / W, W), false, c->stream, true,
                                 (long long)c->ncol * c->ny);
        if (rc) return rc;
        after_sweep(c);
        return IBLB_OK;
    }
    int rc = join_comm(c);  // boundary columns of the current state (comm stream)
    if (rc) return rc;
    if (!c->send_sweep) {  // the send buffers hold the one-step (or IB) halo: pack the 2-step one
        HIP_TRY(c, launch_pack_sweep_halo<T>(gptr<T>(c, c->cur), c->L, (T*)c->send_left, (T*)c->send_right,
                                             c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
    }
    const bool ov = c->overlap;
    hipStream_t bs = ov ? c->comm_stream : c->stream;
    const int ni = c->ncol - 4;  // interior [2, ncol-2): needs nothing from the halo
    if (ov && c->sweep_order == 1) {
        // the same dependencies, submitted interior first: the launch the step time depends on
        // leaves the host before the RCCL group and the boundary launch (whose host cost then
        // overlaps the interior); boundary(t) waits for ev_pre = the compute work before
        // interior(t), i.e. interior(t-2), which read the columns it overwrites
        HIP_TRY(c, hipEventRecord(c->ev_pre, c->stream));
        if (ni > 0 && (rc = sweep_launch<T>(c, sweep_args<T>(c, 2, W, c->ncol - 2, (ni + W - 1) / W, W), false,
                                            c->stream, true, (long long)ni * c->ny)))
            return rc;
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        if ((rc = exchange_rccl(c, bs, false, true))) return rc;
        HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_pre, 0));
        if ((rc = sweep_launch<T>(c, sweep_args<T>(c, 0, c->ncol - 2, c->ncol, 2, 2), true, bs, false, 0))) return rc;
        HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
        after_sweep(c);
        c->send_sweep = true;
        c->send_deep = 0;
        return IBLB_OK;
    }
    if (!ov) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_bnd, 0));
    if ((rc = exchange_rccl(c, bs, false, true))) return rc;
    if (ov) HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_int, 0));
    // boundary sweeps: [0, 2) and [ncol-2, ncol)
    if ((rc = sweep_launch<T>(c, sweep_args<T>(c, 0, c->ncol - 2, c->ncol, 2, 2), true, bs, false, 0))) return rc;
    if (ov) HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
    if (ni > 0 && (rc = sweep_launch<T>(c, sweep_args<T>(c, 2, W, c->ncol - 2, (ni + W - 1) / W, W), false, c->stream,
                                        true, (long long)ni * c->ny)))
        return rc;
    if (ov) HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
    else {
        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
    }
    after_sweep(c);
    c->send_sweep = true;
    c->send_deep = 0;
    return IBLB_OK;
}

// One reference iteration for a context whose halo (if any) and force^t are in place.
int advance(iblb_ctx* c) {
    int rc;
    const bool f64 = c->prec == IBLB_PREC_F64;
    if (c->phase == PH_BOOT) {
        rc = f64 ? launch_boot_step<double>(c) : launch_boot_step<float>(c);
        if (rc) return rc;
        c->phase = PH_RUN;
    } else {
        rc = f64 ? launch_fused_step<double>(c, 0, c->ncol) : launch_fused_step<float>(c, 0, c->ncol);
        if (rc) return rc;
    }
    if (rccl_multi(c)) {  // the whole state was written on the compute stream
        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
    }
    after_step(c);
    return IBLB_OK;
}

int check_ready(iblb_ctx* c) {
    if (c->phase == PH_EMPTY) return fail(c, IBLB_ERR_STATE, "no state: call iblb_set_state first");
    if (!single_slab(c) && c->transport == TR_NONE)
        return fail(c, IBLB_ERR_STATE, "slab context is not linked to its neighbours");
    return IBLB_OK;
}

// Cilia kinematics of iteration it = c->t into the Lagrangian arrays (main.cu:822-841).
// Any force still owed to the previous points must have been evaluated before.
int run_cilia(iblb_ctx* c) {
    const iblb_cilia& k = c->cilia;
    const int it = (int)c->t;
    HIP_TRY(c, launch_define_filament(k.T, it, k.c_space, k.p_step, (double)k.c_num, c->cil_samples, c->cil_lasts,
                                      c->cil_bpoints, c->stream));
    HIP_TRY(c, launch_boundary_check(k.c_space, k.c_num, c->nx, it, c->cil_bpoints, c->d_s, c->d_us, c->d_eps,
                                     c->stream));
    c->ns = CILIA_POINTS * k.c_num;
    return IBLB_OK;
}

int step_one(iblb_ctx* c) {
    int rc = join_comm(c);
    if (rc) return rc;
    if (c->cilia_on) {
        if (c->phase == PH_RUN) {
            if ((rc = ensure_halo(c))) return rc;
            if ((rc = ensure_force(c))) return rc;
        }
        if ((rc = run_cilia(c))) return rc;
    } else if (c->phase == PH_RUN && rccl_multi(c) && c->overlap && c->ib_state == IB_PENDING && !c->halo_valid &&
               c->ncol >= 9 && env_long("IBLB_IB_OVERLAP", 1)) {
        const int next = c->sch_n > 0 && sched_entry(c, c->t) != c->sch_cur ? sched_entry(c, c->t) : -1;
        return c->prec == IBLB_PREC_F64 ? ib_overlapped_step<double>(c, next) : ib_overlapped_step<float>(c, next);
    } else if (c->sch_n > 0 && sched_entry(c, c->t) != c->sch_cur) {
        // the force owed to the previous iteration's points first, then this iteration's points
        if (c->phase == PH_RUN) {
            if ((rc = ensure_halo(c))) return rc;
            if ((rc = ensure_force(c))) return rc;
        }
        if ((rc = sched_use(c, sched_entry(c, c->t)))) return rc;
    }
    if (c->phase == PH_RUN && rccl_multi(c) && c->overlap && !c->halo_valid && c->ib_state != IB_PENDING &&
        c->ncol >= 3)
        return c->prec == IBLB_PREC_F64 ? overlapped_step<double>(c) : overlapped_step<float>(c);
    if (c->phase == PH_RUN) {
        if ((rc = ensure_halo(c))) return rc;
        if ((rc = ensure_force(c))) return rc;
    }
    rc = advance(c);
    if (rc) return rc;
    if (c->phase == PH_RUN && c->t == 1 && c->rho0) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        free_boot(c);
    }
    return IBLB_OK;
}

size_t round_up(size_t v, size_t m) { return (v + m - 1) / m * m; }

// Allocation zeroed on the context's (non-blocking) stream, so later work on that stream is
// ordered after the clear.
int alloc_zero(iblb_ctx* c, void** p, size_t bytes) {
    HIP_TRY(c, hipMalloc(p, bytes));
    HIP_TRY(c, hipMemsetAsync(*p, 0, bytes, c->stream));
    return IBLB_OK;
}

// Scratch device buffer freed at scope exit.
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
};

// Make halos and force^t of the current state available to a reader.
int prepare_read(iblb_ctx* c) {
    int rc = check_ready(c);
    if (rc) return rc;
    if (c->phase != PH_RUN) return IBLB_OK;
    if ((rc = join_comm(c))) return rc;
    if (c->transport == TR_LOCAL) {
        if (!c->halo_valid || c->ib_state == IB_PENDING)
            return fail(c, IBLB_ERR_STATE, "local group state not prepared (use iblb_group_step)");
        return IBLB_OK;
    }
    if ((rc = ensure_halo(c))) return rc;
    return ensure_force(c);
}

// rho [N] and u [2N] of the slab in the reference layout (j = y*ncol + xc), into device
// buffers, on the context's stream.  The state must be prepared (prepare_read).
int macro_device(iblb_ctx* c, double* dr, double* du) {
    if (c->phase == PH_BOOT) {
        HIP_TRY(c, launch_field_out(c->rho0, dr, c->L, 1, c->fplane, 0., 0., c->stream));
        HIP_TRY(c, launch_field_out(c->u0, du, c->L, 2, c->fplane, 0., 0., c->stream));
        return IBLB_OK;
    }
    const double* fd = c->ib_state == IB_READY ? c->fdense : nullptr;
    if (c->prec == IBLB_PREC_F64)
        HIP_TRY(c, launch_macro_out<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), fd, c->fplane,
                                            c->coef.gx, c->coef.gy, dr, du, c->stream));
    else
        HIP_TRY(c, launch_macro_out<float>(gptr<float>(c, c->cur), c->L, halo_of<float>(c, c->cur), fd, c->fplane,
                                           c->coef.gx, c->coef.gy, dr, du, c->stream));
    return IBLB_OK;
}

}  // namespace

// ============================================================================================
extern "C" {

const char* iblb_version(void) { return "iblb-mi355x 0.1 (gfx950)"; }

int iblb_device_count(int* n) {
    if (!n) return IBLB_ERR_ARG;
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
    *n = k;
    return IBLB_OK;
}

int iblb_config_default(iblb_config* cfg) {
    if (!cfg) return IBLB_ERR_ARG;
    std::memset(cfg, 0, sizeof(*cfg));
    // main.cu:267-321 with the default arguments c_num=6, c_space=48, Re=1, T=1e5
    cfg->nx = 288;
    cfg->ny = 192;
    const double SPEED = 0.8 * 1000 / 100000.;
    const double cs = 0.577;  // main.cu:27
    cfg->tau = (SPEED * 96) / (1.0 * cs * cs) + 1. / 2.;
    cfg->tau2 = 1. / (12. * (cfg->tau - (1. / 2.))) + (1. / 2.);
    cfg->precision = IBLB_PREC_F64;
    cfg->flux_norm = 192.;
    cfg->flux_column = cfg->nx - 5;
    cfg->device = 0;
    cfg->x_begin = 0;
    cfg->x_count = 0;
    cfg->max_points = 0;
    return IBLB_OK;
}

const char* iblb_last_error(const iblb_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int iblb_create(const iblb_config* cfg, iblb_ctx** out) {
    if (!cfg || !out) return fail(nullptr, IBLB_ERR_ARG, "null argument");
    *out = nullptr;
    if (cfg->nx < 1 || cfg->ny < 2) return fail(nullptr, IBLB_ERR_ARG, "need nx >= 1 and ny >= 2");
    if (!(cfg->tau > 0.5) || !(cfg->tau2 > 0.5)) return fail(nullptr, IBLB_ERR_ARG, "need tau, tau2 > 0.5");
    if (cfg->precision != IBLB_PREC_F64 && cfg->precision != IBLB_PREC_F32)
        return fail(nullptr, IBLB_ERR_ARG, "precision must be IBLB_PREC_F64 or IBLB_PREC_F32");
    if (cfg->flux_norm == 0.) return fail(nullptr, IBLB_ERR_ARG, "flux_norm must be non-zero");
    const int xb = cfg->x_count > 0 ? cfg->x_begin : 0;
    const int nc = cfg->x_count > 0 ? cfg->x_count : cfg->nx;
    if (xb < 0 || xb + nc > cfg->nx) return fail(nullptr, IBLB_ERR_ARG, "slab outside the lattice");
    if (cfg->max_points < 0) return fail(nullptr, IBLB_ERR_ARG, "max_points < 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, IBLB_ERR_NODEVICE, "no HIP device visible (the HIP path has no CPU fallback)");
    if (cfg->device < 0 || cfg->device >= ndev) return fail(nullptr, IBLB_ERR_ARG, "device ordinal out of range");

    iblb_ctx* c = new iblb_ctx();
    c->cfg = *cfg;
    c->nx = cfg->nx;
    c->ny = cfg->ny;
    c->x_begin = xb;
    c->ncol = nc;
    c->prec = cfg->precision;
    c->esize = c->prec == IBLB_PREC_F64 ? 8 : 4;
    c->V = c->prec == IBLB_PREC_F64 ? vec_of<double>() : vec_of<float>();
    c->nch = chunks_per_column(c->ny, c->V);
    c->device = cfg->device;
    c->max_points = cfg->max_points;
    // collide-stream variant measured fastest on MI355X (scripts/tune_fused.py, profiles/) with
    // the interleaved layout: f64 = DPP row shift + nontemporal stores (5), f32 = nontemporal
    // loads and stores (3; 0.193 ms vs 0.218 ms planar variant 2, profiles/r01e_tune_f32.log)
    c->variant = (int)env_long("IBLB_FUSED_VARIANT", c->prec == IBLB_PREC_F64 ? 5 : 3);
    c->sweep_on = env_long("IBLB_SWEEP", 1) != 0;
    // measured on MI355X (profiles/r01p_tune_*.log, r01q_*, r01s_*, r01t_*): 16 B per lane (f64 2
    // cells, f32 4), short sweeps (f64 4 columns: 4096^2 0.227 ms/iteration vs 0.406 one-step,
    // 512 x 4096 0.034 vs 0.061; f32 6 columns: 0.118 vs 0.199), nontemporal stores, the linear
    // wave order dealt to the XCDs in contiguous ranges (map 2, 4 % faster than plain linear) with
    // alternate sweeps walking towards each other (alt: HBM fetch 1.08x the state instead of
    // 1.38x / 1.60x); the XCD-contiguous 4-sweep workgroups (map 0) measured 10-15 % slower
    c->sweep_w = (int)env_long("IBLB_SWEEP_W", c->prec == IBLB_PREC_F64 ? 4 : 6);
    c->sweep_vs = (int)env_long("IBLB_SWEEP_VS", c->prec == IBLB_PREC_F64 ? 2 : 4);
    c->sweep_variant = (int)env_long("IBLB_SWEEP_VARIANT", 1);
    c->sweep_map = (int)env_long("IBLB_SWEEP_MAP", 2);
    c->sweep_alt = (int)env_long("IBLB_SWEEP_ALT", 1);
    // deep sweeps (K = 3 .. 6 iterations per launch), measured on MI355X at 4096^2
    // (profiles/r01d5_tune_deep_*.log, r01g_tune_*.log): f64 K = 5, 2 cells per lane, ~96-column
    // sweeps 0.133 ms/iteration (126k MLUPS; K = 2: 0.236, one-step 0.399); f32 K = 5, 2 cells
    // per lane, ~64 columns 0.087 (193k; K = 2: 0.121).  Widths are balanced to whole rounds of
    // resident waves.
    c->sweep_depth = (int)env_long("IBLB_SWEEP_DEPTH", 5);
    if (c->sweep_depth > 6) c->sweep_depth = 6;
    c->deep_w = (int)env_long("IBLB_DEEP_W", c->prec == IBLB_PREC_F64 ? 96 : 64);
    c->deep_vs = (int)env_long("IBLB_DEEP_VS", 2);
    c->deep_variant = (int)env_long("IBLB_DEEP_VARIANT", 1);
    c->deep_balance = (int)env_long("IBLB_DEEP_BALANCE", 1);
    // slabs of an RCCL group: one cell per lane (self ring 512 / 1024 / 2048 x 4096: 0.0347 /
    // 0.0542 / 0.0935 ms/iteration vs 0.0380 / 0.0568 / 0.0942 with two, profiles/r01e7_*)
    c->deep_slab_vs = (int)env_long("IBLB_DEEP_SLAB_VS", 1);
    c->deep_bnd_vs = (int)env_long("IBLB_DEEP_BND_VS", c->deep_slab_vs);
    if (c->cfg.flux_column < 0) c->cfg.flux_column = c->nx - 5;

    const double tau = cfg->tau, tau2 = cfg->tau2, cs = 0.57735;
    c->coef.omega_p = 1. / tau;
    c->coef.omega_m = 1. / tau2;
    c->coef.kguo = 1. - 1. / (2. * tau);
    c->coef.inv_cs2 = 1. / (cs * cs);
    c->coef.inv_cs4 = 1. / (cs * cs * cs * cs);
    c->coef.inv_2cs2 = 1. / (2 * cs * cs);
    c->coef.inv_2cs4 = 1. / (2 * cs * cs * cs * cs);
    c->coef.gx = cfg->body_force[0];
    c->coef.gy = cfg->body_force[1];
    c->kc = make_kconst(c->coef);

    auto bail = [&](int rc) { g_create_error = c->err; iblb_destroy(c); return rc; };
    if (hipSetDevice(c->device) != hipSuccess) return bail(fail(c, IBLB_ERR_HIP, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(c, IBLB_ERR_HIP, "hipStreamCreate failed"));

    // slab layout: a column of a plane holds `rows` = ny rounded up to whole waves.
    //  interleaved (default, IBLB_LAYOUT=1): g[xc*col + k*plane + y], the 9 planes of a
    //    column adjacent (plane = rows + IBLB_PLANE_PAD, col = 9*plane + IBLB_COL_PAD);
    //    4096^2 f64: 0.398 ms vs 0.425 ms planar (profiles/r01d_tune_layout_f64.log)
    //  planar (IBLB_LAYOUT=0): g[k*plane + xc*rows + y], planes padded apart so the 9 read and
    //    9 write streams do not start on the same HBM channel (a zero pad costs ~15 %,
    //    profiles/r01_tune_*.log)
    const bool f64 = c->prec == IBLB_PREC_F64;
    const long rows = (long)round_up((size_t)c->ny, (size_t)(64 * c->V));
    const bool interleaved = env_long("IBLB_LAYOUT", 1) == 1;
    c->L.ny = c->ny;
    c->L.ncol = c->ncol;
    c->L.rows = rows;
    long buf;  // elements of one population buffer
    if (interleaved) {
        c->L.plane = rows + env_long("IBLB_PLANE_PAD", 0);
        c->L.col = 9 * c->L.plane + env_long("IBLB_COL_PAD", f64 ? 64 : 0);
        buf = (long)c->ncol * c->L.col;
    } else {
        c->L.col = rows;
        c->L.plane = (long)c->ncol * rows + env_long("IBLB_PLANE_PAD", f64 ? 256 : 1024);
        buf = 9 * c->L.plane;
    }
    c->fplane = (long)c->ncol * rows;
    // buffer 1 starts `gap` elements after the end of buffer 0
    const long gap = env_long("IBLB_BUF_GAP", c->prec == IBLB_PREC_F64 ? 320 : 0);
    const size_t gbytes = (size_t)(2 * buf + gap + 2 * GUARD) * c->esize;
    {
        int rc = alloc_zero(c, (void**)&c->g_alloc, gbytes);
        if (rc) return bail(rc);
        c->g[0] = c->g_alloc + GUARD * c->esize;
        c->g[1] = c->g_alloc + (GUARD + buf + gap) * c->esize;
        c->buf_elems = buf;
        c->buf_gap = gap;
    }
    c->band_on = (int)env_long("IBLB_IB_BAND", 1);
    c->band_fused = (int)env_long("IBLB_BAND_FUSED", 0);
    c->band_full = (int)env_long("IBLB_BAND_FULL", 1);
    c->band_hosttab = (int)env_long("IBLB_BAND_HOSTTAB", 1);
    c->band_tail_ds = (int)env_long("IBLB_BAND_TAIL_DS", 1);
    // halo buffers: recv_left, recv_right, send_left, send_right; each 10 (2-step) or 21 (IB)
    // slots + guards
    {
        c->halo_slots = c->max_points > 0 ? IB_HALO_SLOTS : SWEEP_HALO_SLOTS;
        if (c->sweep_depth >= 3) c->halo_slots = std::max(c->halo_slots, deep_slots(c->sweep_depth));
        const size_t slot = (size_t)(c->halo_slots * rows + 2 * GUARD) * c->esize;
        int rc = alloc_zero(c, (void**)&c->halo_alloc, 4 * slot);
        if (rc) return bail(rc);
        c->recv_left = c->halo_alloc + 0 * slot + GUARD * c->esize;
        c->recv_right = c->halo_alloc + 1 * slot + GUARD * c->esize;
        c->send_left = c->halo_alloc + 2 * slot + GUARD * c->esize;
        c->send_right = c->halo_alloc + 3 * slot + GUARD * c->esize;
    }
    int rc = alloc_zero(c, (void**)&c->d_Q, 4 * sizeof(double));
    if (rc) return bail(rc);
    if (c->max_points > 0) {
        const size_t np = (size_t)c->max_points;
        if ((rc = alloc_zero(c, (void**)&c->d_s, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_us, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_Fs, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_eps, np * sizeof(int)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_Fs_sum, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->fdense, 2 * (size_t)c->fplane * sizeof(double)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->flags, (size_t)c->ncol * c->nch))) return bail(rc);
    }
    *out = c;
    return IBLB_OK;
}

void iblb_destroy(iblb_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    for (hipStream_t st : {c->band_st, c->deep_st})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    for (hipEvent_t e : {c->ev_b0, c->ev_b1, c->ev_b2, c->ev_bd})
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < 4; ++i) {
        if (c->band_pin_ev[i]) (void)hipEventDestroy(c->band_pin_ev[i]);
        if (c->band_pin[i]) (void)hipHostFree(c->band_pin[i]);
    }
    if (c->ev_bnd) (void)hipEventDestroy(c->ev_bnd);
    if (c->ev_int) (void)hipEventDestroy(c->ev_int);
    if (c->ev_pre) (void)hipEventDestroy(c->ev_pre);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->g_alloc) (void)hipFree(c->g_alloc);
    void* bufs[] = {c->cil_samples, c->cil_lasts, c->cil_bpoints, c->s_alloc, c->d_band,
                    c->halo_alloc, c->rho0, c->u0, c->force0, c->d_s, c->d_us, c->d_Fs,
                    c->d_eps, c->d_Fs_sum, c->fdense, c->flags, c->d_Q, c->d_sch_s, c->d_sch_us, c->d_sch_eps};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->left && c->left->right == c) c->left->right = nullptr;
    if (c->right && c->right->left == c) c->right->left = nullptr;
    delete c;
}

int iblb_set_state(iblb_ctx* c, const double* rho, const double* u, const double* f, const double* force) {
    if (!c) return IBLB_ERR_ARG;
    c->deep_chain = false;  // the state is rewritten: no deep cycle chain across this
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const long N = (long)c->ncol * c->ny;
    const size_t nb = (size_t)N * sizeof(double);
    free_boot(c);
    int rc;
    if ((rc = alloc_zero(c, (void**)&c->rho0, (size_t)c->fplane * sizeof(double)))) return rc;
    if ((rc = alloc_zero(c, (void**)&c->u0, 2 * (size_t)c->fplane * sizeof(double)))) return rc;
    if ((rc = alloc_zero(c, (void**)&c->force0, 2 * (size_t)c->fplane * sizeof(double)))) return rc;

    DevBuf d_rho, d_u, d_force, d_f, d_F;
    HIP_TRY(c, hipMalloc(&d_rho.p, nb));
    HIP_TRY(c, hipMalloc(&d_u.p, 2 * nb));
    HIP_TRY(c, hipMalloc(&d_force.p, 2 * nb));
    if (rho) {
        HIP_TRY(c, hipMemcpy(d_rho.p, rho, nb, hipMemcpyHostToDevice));
    } else {
        std::vector<double> ones((size_t)N, 1.0);  // RHO_0 (main.cu:28, 638)
        HIP_TRY(c, hipMemcpy(d_rho.p, ones.data(), nb, hipMemcpyHostToDevice));
    }
    if (u) HIP_TRY(c, hipMemcpy(d_u.p, u, 2 * nb, hipMemcpyHostToDevice));
    else HIP_TRY(c, hipMemsetAsync(d_u.p, 0, 2 * nb, c->stream));
    if (force) HIP_TRY(c, hipMemcpy(d_force.p, force, 2 * nb, hipMemcpyHostToDevice));
    else HIP_TRY(c, hipMemsetAsync(d_force.p, 0, 2 * nb, c->stream));
    HIP_TRY(c, hipMalloc(&d_f.p, 9 * nb));
    if (f) {
        HIP_TRY(c, hipMemcpy(d_f.p, f, 9 * nb, hipMemcpyHostToDevice));
    } else {
        // main.cu:720-754: f = f0 = equilibrium(u, rho) with force 0
        DevBuf zero;
        HIP_TRY(c, hipMalloc(&d_F.p, 9 * nb));
        HIP_TRY(c, hipMalloc(&zero.p, 2 * nb));
        HIP_TRY(c, hipMemsetAsync(zero.p, 0, 2 * nb, c->stream));
        rc = iblb_equilibrium((const double*)d_u.p, (const double*)d_rho.p, (double*)d_f.p, (const double*)zero.p,
                              (double*)d_F.p, c->ncol, c->ny, c->cfg.tau, c->stream);
        if (rc) return fail(c, rc, "initial equilibrium launch failed");
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    if (c->prec == IBLB_PREC_F64)
        HIP_TRY(c, launch_pop_in<double>((const double*)d_f.p, gptr<double>(c, c->cur), c->L, c->stream));
    else
        HIP_TRY(c, launch_pop_in<float>((const double*)d_f.p, gptr<float>(c, c->cur), c->L, c->stream));
    HIP_TRY(c, launch_field_in((const double*)d_rho.p, c->rho0, c->L, 1, c->fplane, c->stream));
    HIP_TRY(c, launch_field_in((const double*)d_u.p, c->u0, c->L, 2, c->fplane, c->stream));
    HIP_TRY(c, launch_field_in((const double*)d_force.p, c->force0, c->L, 2, c->fplane, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_Q, 0, 4 * sizeof(double), c->stream));
    if (c->fdense) {
        HIP_TRY(c, hipMemsetAsync(c->fdense, 0, 2 * (size_t)c->fplane * sizeof(double), c->stream));
        HIP_TRY(c, hipMemsetAsync(c->flags, 0, (size_t)c->ncol * c->nch, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->cilia_on) {  // the beat restarts with the state (lasts = 0, main.cu:348-359)
        int rc2 = reset_cilia_state(c);
        if (rc2) return rc2;
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    c->phase = PH_BOOT;
    c->t = 0;
    c->ib_state = IB_NONE;
    c->halo_valid = false;
    return IBLB_OK;
}

}  // extern "C"

// Streams of the overlapped band cycle: the band chain on band_st restricted to `band_reserve`
// CUs (the top mask bits of the CUs the cycle may use: bit i is a CU of XCD i % 8, so 8m bits are
// m CUs of every XCD, profiles/r02n_xcc_probe.txt), the cycle's deep sweep on deep_st masked to
// the others.  A lone slab may use the whole chip; a slab of an RCCL group the compute stream's
// CUs (comp_mask: the comm stream keeps its reserved CUs for the exchange and the boundary
// sweeps).  The context's stream is never replaced: it keeps its CUs for every other launch and
// joins the two with events in band_step.  Defaults: the fused band kernel (one workgroup per
// patch) gets 8 * ceil(patches / (8 * IBLB_BAND_ROUNDS)) CUs (rounds of one workgroup per CU);
// the launch-per-level chain one XCD's worth, two where the trapezoids hold more than 5 % of the
// cycle's lattice updates (one-step launches, HBM-bound; the deep sweep is issue-bound).
// IBLB_BAND_RESERVE_CUS overrides; 0: both on the context's stream, in sequence.
static int band_streams(iblb_ctx* c, long long band_lu, long long deep_lu, int npatch) {
    const bool slab = rccl_multi(c);
    if (c->transport == TR_LOCAL || (!slab && c->comm_stream) || (slab && env_long("IBLB_BAND_SLAB_OV", 1) == 0))
        return IBLB_OK;
    if (!c->ncu) {
        hipDeviceProp_t prop;
        HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
        c->ncu = prop.multiProcessorCount;
    }
    const int per_xcd = std::max(1, c->ncu / 8);
    long dflt;
    if (c->band_fused) {
        const long rounds = std::max(1L, env_long("IBLB_BAND_ROUNDS", 2));
        dflt = 8 * ((npatch + 8 * rounds - 1) / (8 * rounds));
    } else {
        const double share = (double)band_lu / (double)std::max(1LL, band_lu + (long long)c->sweep_depth * deep_lu);
        dflt = (share > 0.05 ? 2 : 1) * per_xcd;
    }
    // the CUs the cycle may use
    std::vector<uint32_t> base((size_t)(c->ncu + 31) / 32, 0u);
    int avail = 0;
    for (int i = 0; i < c->ncu; ++i)
        if (!slab || c->comp_mask.empty() || (c->comp_mask[(size_t)i / 32] >> (i % 32) & 1u)) {
            base[(size_t)i / 32] |= 1u << (i % 32);
            ++avail;
        }
    long want = env_long("IBLB_BAND_RESERVE_CUS", dflt);
    if (want < 0 || want >= avail) want = 0;
    if (want == c->band_reserve || (c->band_sticky && c->band_st)) return IBLB_OK;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (hipStream_t* st : {&c->band_st, &c->deep_st})
        if (*st) {
            HIP_TRY(c, hipStreamSynchronize(*st));
            (void)hipStreamDestroy(*st);
            *st = nullptr;
        }
    if (want) {
        std::vector<uint32_t> deep(base.size(), 0u), band(base.size(), 0u);
        long taken = 0;
        for (int i = c->ncu - 1; i >= 0; --i) {
            if (!(base[(size_t)i / 32] >> (i % 32) & 1u)) continue;
            std::vector<uint32_t>& m = taken < want ? band : deep;
            m[(size_t)i / 32] |= 1u << (i % 32);
            ++taken;
        }
        HIP_TRY(c, hipExtStreamCreateWithCUMask(&c->deep_st, (uint32_t)deep.size(), deep.data()));
        HIP_TRY(c, hipExtStreamCreateWithCUMask(&c->band_st, (uint32_t)band.size(), band.data()));
        for (hipEvent_t* e : {&c->ev_b0, &c->ev_b1, &c->ev_b2, &c->ev_bd})
            if (!*e) HIP_TRY(c, hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventDisableSystemFence));
    }
    c->band_reserve = (int)want;
    return IBLB_OK;
}

// IB band plan for band_step from the x coordinates of every point the cycles may see (host
// copy: the static points, or every entry of a schedule plus the points before it); band_valid
// stays false where the cycle does not apply (see band_ready) or does not pay (bands over half
// the lattice, bands within 2(K-1) columns of the lattice edge: the reference's flat-index wrap).
template <typename T>
static int plan_bands_t(iblb_ctx* c, const std::vector<float>& xy) {
    const int K = c->sweep_depth, R = 2 * (K - 1);
    // A slab of an RCCL group: local columns, bands and gaps inside [K, ncol-K).  Every rank
    // holds every point and tests every point against its own slab's interior, so all ranks take
    // the same decision (the cycle's deep-halo exchange is collective).
    const bool slab = !single_slab(c);
    const int nx = slab ? c->ncol : c->nx;  // local columns
    const int lo = slab ? K : 0, hi = slab ? c->ncol - K : c->nx;
    const int ny = c->ny;
    // forced cells of every point: columns [x0-1, x0+1] x rows [y0-1, y0+1] (the 3x3 nodes; rows
    // outside the lattice receive nothing), as a row range per column
    std::vector<int> fy0((size_t)nx, INT_MAX), fy1((size_t)nx, INT_MIN);
    for (size_t k = 0; k + 1 < xy.size(); k += 2) {
        double x0 = std::nearbyint((double)xy[k]);
        const int y0 = (int)std::nearbyint((double)xy[k + 1]);
        if (slab) {
            int r = -1;
            for (size_t q = 0; q < c->slab_begin.size(); ++q)
                if (x0 >= c->slab_begin[q] && x0 < c->slab_begin[q] + c->slab_count[q]) r = (int)q;
            const double b = r >= 0 ? c->slab_begin[(size_t)r] : 0., e = r >= 0 ? b + c->slab_count[(size_t)r] : 0.;
            if (r < 0 || !(x0 - 1 - R >= b + K && x0 + 1 + R <= e - 1 - K)) {
                c->band_valid = false;
                return IBLB_OK;
            }
            if (r != c->rank) continue;
            x0 -= c->x_begin;
        } else if (!(x0 - 1 - R >= 0. && x0 + 1 + R <= nx - 1.)) {
            c->band_valid = false;
            return IBLB_OK;
        }
        // (clamped into the lattice: a point whose nodes all miss it still gets a patch, so the
        // fused band kernel, which lists points by patch, writes its F_s)
        const int ya = std::min(std::max(0, y0 - 1), ny - 1), yb = std::max(std::min(ny - 1, y0 + 1), 0);
        for (int x = (int)x0 - 1; x <= (int)x0 + 1; ++x) {
            fy0[(size_t)x] = std::min(fy0[(size_t)x], std::min(ya, yb));
            fy1[(size_t)x] = std::max(fy1[(size_t)x], std::max(ya, yb));
        }
    }
    // forced column intervals with their row range, merged into patches {x0, x1, y0, y1} whose
    // trapezoids stay apart (gaps >= R + 8 columns)
    std::vector<std::array<int, 4>> b;
    for (int x = 0; x < nx;) {
        if (fy0[(size_t)x] > fy1[(size_t)x]) { ++x; continue; }
        std::array<int, 4> iv{x, x, fy0[(size_t)x], fy1[(size_t)x]};
        while (iv[1] + 1 < nx && fy0[(size_t)iv[1] + 1] <= fy1[(size_t)iv[1] + 1]) {
            ++iv[1];
            iv[2] = std::min(iv[2], fy0[(size_t)iv[1]]);
            iv[3] = std::max(iv[3], fy1[(size_t)iv[1]]);
        }
        if (!b.empty() && iv[0] - b.back()[1] - 1 < 2 * R + 8) {
            b.back()[1] = iv[1];
            b.back()[2] = std::min(b.back()[2], iv[2]);
            b.back()[3] = std::max(b.back()[3], iv[3]);
        } else {
            b.push_back(iv);
        }
        x = iv[1] + 1;
    }
    if (c->band_valid && b == c->band_b) return IBLB_OK;  // the installed plan covers these points
    c->band_valid = false;
    // Rows: a patch's output rows are its forced rows +- (K-1), widened to whole row chunks of
    // the deep sweep (which advances the rest of the patch's columns); IBLB_BAND_ROWS=0: whole
    // columns (the trapezoid then covers every row, as before patches)
    int nchd = 0;
    (void)sweepk_geometry<T>(K, c->deep_vs, c->deep_variant, false, ny, &nchd);
    const int vsd = c->deep_vs, gd = (K - 1 + vsd - 1) / vsd, rpc = (64 - 2 * gd) * vsd;  // deep rows per chunk
    if (nchd <= 0 || (ny + rpc - 1) / rpc != nchd) return IBLB_OK;
    const bool rows = env_long("IBLB_BAND_ROWS", 1) != 0;
    const int V64 = 64 * c->V;  // rows per chunk of the one-step kernel
    std::vector<std::array<int, 4>> pr(b.size());  // per patch: deep chunks [ca, cb), rows [ya, yb)
    for (size_t q = 0; q < b.size(); ++q) {
        const int ca = rows ? std::max(0, b[q][2] - (K - 1)) / rpc : 0;
        const int cb = rows ? std::min(ny - 1, b[q][3] + (K - 1)) / rpc + 1 : nchd;
        pr[q] = {ca, cb, ca * rpc, std::min(ny, cb * rpc)};
    }
    // the trapezoid: level j covers the patch +- (K-1-j) more columns and rows than its output
    std::vector<int> tab;
    std::vector<int> off((size_t)K), cnt((size_t)K), nchl((size_t)K, 0);
    // the fused band kernel's patch table (BandArgs::pt): x0 range of the patch's points, then per
    // level {first entry (ints into d_band), entries, chunks per entry}
    std::vector<int> ptab(b.size() * BAND_PT, 0);
    for (size_t q = 0; q < b.size(); ++q) {
        ptab[q * BAND_PT + 0] = b[q][0] + 1;
        ptab[q * BAND_PT + 1] = b[q][1] - 1;
    }
    long long band_lu = 0;
    for (int j = 0; j < K; ++j) {
        off[j] = (int)tab.size();
        cnt[j] = 0;
        const int m = K - 1 - j;
        for (size_t q = 0; q < b.size(); ++q) {
            const int ylo = std::max(0, pr[q][2] - m), yhi = std::min(ny, pr[q][3] + m);
            const int ch0 = ylo / V64, ch1 = std::min(c->nch, (yhi + V64 - 1) / V64);
            nchl[j] = std::max(nchl[j], ch1 - ch0);
            ptab[q * BAND_PT + 2 + 3 * j] = (int)tab.size();
            ptab[q * BAND_PT + 3 + 3 * j] = b[q][1] - b[q][0] + 1 + 2 * (R - j);
            ptab[q * BAND_PT + 4 + 3 * j] = ch1 - ch0;
            for (int x = b[q][0] - R + j; x <= b[q][1] + R - j; ++x) {
                tab.insert(tab.end(), {x, ch0, ch1, pr[q][2], pr[q][3]});
                ++cnt[j];
                band_lu += (long long)(ch1 - ch0) * V64;
            }
        }
    }
    if (!slab && 2 * band_lu > (long long)K * nx * ny) return IBLB_OK;  // (a slab: the same decision on every rank)
    // the deep sweep: every column farther than K-1 from the forced columns (the gaps), and the
    // patches' output columns outside their rows; regions of (columns, deep chunks)
    struct Region { int x0, x1, c0, c1; };
    std::vector<Region> reg;
    int prev = lo;
    for (size_t q = 0; q < b.size(); ++q) {
        const int bx0 = b[q][0] - (K - 1), bx1 = b[q][1] + K;  // output columns [bx0, bx1)
        if (bx0 > prev) reg.push_back({prev, bx0, 0, nchd});
        if (pr[q][0] > 0) reg.push_back({bx0, bx1, 0, pr[q][0]});
        if (pr[q][1] < nchd) reg.push_back({bx0, bx1, pr[q][1], nchd});
        prev = bx1;
    }
    if (prev < hi) reg.push_back({prev, hi, 0, nchd});
    double work = 0.;  // in whole-column equivalents
    long long deep_lu = 0;
    for (auto& g : reg) {
        work += (double)(g.x1 - g.x0) * (g.c1 - g.c0) / nchd;
        deep_lu += (long long)(g.x1 - g.x0) * std::min(ny, (g.c1 - g.c0) * rpc);
    }
    int rc = band_streams(c, band_lu / std::max(1, ny), deep_lu / std::max(1, ny), (int)b.size());
    if (rc) return rc;
    // sweeps of ~deep_w columns, balanced to whole rounds of resident waves over the deep
    // sweep's CUs (a sweep over a patch's columns launches every chunk; those of the patch exit)
    const int W = std::max(1, c->deep_w);
    int nch = 0;
    const int wpc = sweepk_geometry<T>(K, c->deep_vs, c->deep_variant, false, c->ny, &nch);
    const int ncu = (slab ? c->ncu - c->reserved_cus : c->ncu) - c->band_reserve;
    long nsw = (long)std::ceil(work / W);
    const long slots = (long)wpc * ncu;
    if (c->deep_balance && slots > 0 && nch > 0 && work > 0.) {
        const long rounds = std::max(1L, (nsw * nch + slots / 2) / slots);
        nsw = std::max(1L, rounds * slots / nch);
    }
    const int sweep_off = (int)tab.size();
    int nsweep = 0;
    for (auto& g : reg) {
        const long w = g.x1 - g.x0;
        const double share = (double)w * (g.c1 - g.c0) / nchd / std::max(work, 1e-9);
        long n = std::max(1L, std::lround((double)nsw * share));
        n = std::min(n, w);
        for (long k = 0; k < n; ++k) {
            tab.insert(tab.end(), {g.x0 + (int)(k * w / n), g.x0 + (int)((k + 1) * w / n), g.c0, g.c1});
            ++nsweep;
        }
    }
    const int pt_off = (int)tab.size();
    tab.insert(tab.end(), ptab.begin(), ptab.end());
    if (tab.size() > c->band_cap) {  // grow (rare: sized for the whole lattice at K+1 levels)
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if (c->d_band) (void)hipFree(c->d_band);
        c->d_band = nullptr;
        c->band_cap = 0;
        const size_t cap = std::max(tab.size(), (size_t)5 * (K + 1) * nx + 8 * (size_t)nsw + 64);
        HIP_TRY(c, hipMalloc(&c->d_band, cap * sizeof(int)));
        c->band_cap = cap;
    }
    // in stream order: the previous cycle's launches (which read the old tables) come first,
    // the next cycle's masked streams start after this copy (band_step's ev_b0).  From pinned
    // memory the copy does not make the host wait for the stream (per-cycle plans of moving
    // points would otherwise serialise host and device every cycle).
    if (tab.size() > c->band_pin_cap) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        const size_t cap = std::max(tab.size(), c->band_cap);
        for (int i = 0; i < 4; ++i) {
            if (c->band_pin[i]) (void)hipHostFree(c->band_pin[i]);
            c->band_pin[i] = nullptr;
        }
        c->band_pin_cap = 0;
        for (int i = 0; i < 4; ++i) HIP_TRY(c, hipHostMalloc((void**)&c->band_pin[i], cap * sizeof(int)));
        c->band_pin_cap = cap;
    }
    const int slot = c->band_pin_i;
    c->band_pin_i = (slot + 1) % 4;
    if (c->band_pin_ev[slot]) HIP_TRY(c, hipEventSynchronize(c->band_pin_ev[slot]));
    else HIP_TRY(c, hipEventCreateWithFlags(&c->band_pin_ev[slot], hipEventDisableTiming));
    std::memcpy(c->band_pin[slot], tab.data(), tab.size() * sizeof(int));
    if (c->band_hosttab) {
        // the kernels read the slot itself (device-accessible pinned memory); band_step records
        // the slot's event after each cycle that reads it
        c->band_tab = c->band_pin[slot];
        c->band_pin_cur = slot;
    } else {
        HIP_TRY(c, hipMemcpyAsync(c->d_band, c->band_pin[slot], tab.size() * sizeof(int), hipMemcpyHostToDevice,
                                  c->stream));
        HIP_TRY(c, hipEventRecord(c->band_pin_ev[slot], c->stream));
        c->band_tab = c->d_band;
        c->band_pin_cur = -1;
    }
    if (!c->s_alloc) {  // the trapezoid's scratch levels: two buffers laid out like g
        const size_t bytes = (size_t)(2 * c->buf_elems + c->buf_gap + 2 * GUARD) * c->esize;
        rc = alloc_zero(c, (void**)&c->s_alloc, bytes);
        if (rc) return rc;
        c->sbuf[0] = c->s_alloc + GUARD * c->esize;
        c->sbuf[1] = c->s_alloc + (GUARD + c->buf_elems + c->buf_gap) * c->esize;
    }
    c->band_off = off;
    c->band_n = cnt;
    c->band_sweep_off = sweep_off;
    c->band_nsweep = nsweep;
    c->band_pt_off = pt_off;
    c->band_npatch = (int)b.size();
    c->band_nchl = nchl;
    c->band_deep_lu = deep_lu;
    c->band_lu = band_lu;
    c->band_flux = -1;
    const int fc = c->cfg.flux_column - (slab ? c->x_begin : 0);
    for (auto& iv : b)
        if (fc >= iv[0] - (K - 1) && fc <= iv[1] + (K - 1)) c->band_flux = fc;
    c->band_b = b;
    c->band_valid = true;
    return IBLB_OK;
}

static int plan_bands(iblb_ctx* c, const std::vector<float>& xs) {  // (x, y) pairs
    if (!c->band_on || xs.empty() || c->sweep_depth < 3 || !c->sweep_on || !(single_slab(c) || band_slab_ok(c)) ||
        c->cilia_on) {
        c->band_valid = false;
        return IBLB_OK;
    }
    return c->prec == IBLB_PREC_F64 ? plan_bands_t<double>(c, xs) : plan_bands_t<float>(c, xs);
}

// The band plan of the cycle starting at iteration c->t under a schedule: the forces of its K
// levels come from the points of iterations t-1 .. t+K-2 (the force owed at the start was, or
// will be, evaluated from iteration t-1's points: the points before the schedule if t = t0).
static int plan_cycle(iblb_ctx* c) {
    const int K = c->sweep_depth, ns = c->ns;
    std::vector<float> xs;
    xs.reserve((size_t)(K + 1) * 2 * ns);
    for (long long it = c->t - 1; it <= c->t + K - 2; ++it) {
        if (it < c->sch_t0) {
            xs.insert(xs.end(), c->sch_x_prev.begin(), c->sch_x_prev.end());
            continue;
        }
        const size_t e = (size_t)sched_entry(c, it);
        xs.insert(xs.end(), c->sch_x.begin() + e * 2 * ns, c->sch_x.begin() + (e + 1) * 2 * ns);
    }
    return plan_bands(c, xs);
}
static std::vector<float> x_coords(int ns, const float* s) {  // (x, y) of every point
    return std::vector<float>(s, s + 2 * (size_t)ns);
}

extern "C" {

int iblb_set_lagrangian(iblb_ctx* c, int ns, const float* s, const float* u_s, const int* epsilon) {
    if (!c || ns < 0) return IBLB_ERR_ARG;
    if (ns > c->max_points) return fail(c, IBLB_ERR_ARG, "ns exceeds max_points of the context");
    if (ns > 0 && (!s || !u_s)) return IBLB_ERR_ARG;
    if (c->cilia_on) return fail(c, IBLB_ERR_STATE, "cilia kinematics active: points come from iblb_set_cilia");
    if (ns > 0 && c->ncol != c->nx) {  // a slab of a group evaluates the points spreading into it
        if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
        for (int k = 0; k < ns; ++k) {
            const double x0 = std::nearbyint((double)s[2 * k]);
            if (!(x0 >= 0. && x0 <= (double)c->nx))
                return fail(c, IBLB_ERR_ARG, "slab groups need 0 <= nearbyint(s_x) <= XDIM (main.cu:202-205)");
        }
    }
    HIP_TRY(c, hipSetDevice(c->device));
    // force^t still owed to the old points: evaluate it before they change
    if (c->ib_state == IB_PENDING) {
        if (c->transport == TR_LOCAL)
            return fail(c, IBLB_ERR_STATE, "local group: set points between iblb_group_step calls only");
        int rc = ensure_force(c);
        if (rc) return rc;
    }
    if (ns > 0) {
        HIP_TRY(c, hipMemcpyAsync(c->d_s, s, 2 * (size_t)ns * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->d_us, u_s, 2 * (size_t)ns * sizeof(float), hipMemcpyHostToDevice, c->stream));
        if (epsilon) {
            HIP_TRY(c, hipMemcpyAsync(c->d_eps, epsilon, (size_t)ns * sizeof(int), hipMemcpyHostToDevice, c->stream));
        } else {
            std::vector<int> ones((size_t)ns, 1);
            HIP_TRY(c, hipMemcpyAsync(c->d_eps, ones.data(), (size_t)ns * sizeof(int), hipMemcpyHostToDevice, c->stream));
        }
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    c->ns = ns;
    c->sch_n = 0;  // a schedule given ahead ends here
    c->sch_cur = -1;
    c->band_sticky = false;
    c->band_valid = false;
    return plan_bands(c, x_coords(ns, s));
}

int iblb_set_lagrangian_steps(iblb_ctx* c, int nsteps, int ns, const float* s, const float* u_s, const int* epsilon) {
    if (!c || ns < 0 || nsteps < 1) return IBLB_ERR_ARG;
    if (ns > c->max_points) return fail(c, IBLB_ERR_ARG, "ns exceeds max_points of the context");
    if (ns > 0 && (!s || !u_s)) return IBLB_ERR_ARG;
    if (c->cilia_on) return fail(c, IBLB_ERR_STATE, "cilia kinematics active: points come from iblb_set_cilia");
    const size_t np = (size_t)nsteps * ns;
    if (ns > 0 && c->ncol != c->nx) {
        if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
        for (size_t k = 0; k < np; ++k) {
            const double x0 = std::nearbyint((double)s[2 * k]);
            if (!(x0 >= 0. && x0 <= (double)c->nx))
                return fail(c, IBLB_ERR_ARG, "slab groups need 0 <= nearbyint(s_x) <= XDIM (main.cu:202-205)");
        }
    }
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->ib_state == IB_PENDING) {  // the force owed to the points before the schedule
        if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: set points between group steps");
        int rc = ensure_force(c);
        if (rc) return rc;
    }
    // host copies for the per-cycle band plans: every entry's x, and the points before the
    // schedule (a force evaluated from them is owed to the first iteration)
    c->sch_x_prev.clear();
    if (c->ns > 0 && c->ib_state == IB_READY) {
        std::vector<float> old(2 * (size_t)c->ns);
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        HIP_TRY(c, hipMemcpy(old.data(), pts_s(c), old.size() * sizeof(float), hipMemcpyDeviceToHost));
        c->sch_x_prev = x_coords(c->ns, old.data());
    }
    if (ns > 0) {
        if ((size_t)nsteps > c->sch_cap || ns != c->ns) {
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            for (void* p : {(void*)c->d_sch_s, (void*)c->d_sch_us, (void*)c->d_sch_eps})
                if (p) (void)hipFree(p);
            c->d_sch_s = c->d_sch_us = nullptr;
            c->d_sch_eps = nullptr;
            c->sch_cap = 0;
            const size_t cap = (size_t)nsteps * c->max_points;
            HIP_TRY(c, hipMalloc(&c->d_sch_s, 2 * cap * sizeof(float)));
            HIP_TRY(c, hipMalloc(&c->d_sch_us, 2 * cap * sizeof(float)));
            HIP_TRY(c, hipMalloc(&c->d_sch_eps, cap * sizeof(int)));
            c->sch_cap = (size_t)nsteps;
        }
        HIP_TRY(c, hipMemcpyAsync(c->d_sch_s, s, 2 * np * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->d_sch_us, u_s, 2 * np * sizeof(float), hipMemcpyHostToDevice, c->stream));
        if (epsilon) {
            HIP_TRY(c, hipMemcpyAsync(c->d_sch_eps, epsilon, np * sizeof(int), hipMemcpyHostToDevice, c->stream));
        } else {
            std::vector<int> ones(np, 1);
            HIP_TRY(c, hipMemcpyAsync(c->d_sch_eps, ones.data(), np * sizeof(int), hipMemcpyHostToDevice, c->stream));
        }
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->sch_x = x_coords((int)np, s);
    }
    c->ns = ns;
    c->sch_t0 = c->t;
    c->sch_n = ns > 0 ? nsteps : 0;
    c->sch_cur = -1;  // d_s still holds the points before the schedule (their force is READY)
    c->band_sticky = true;
    c->band_valid = false;  // planned per cycle (plan_cycle)
    return IBLB_OK;
}

static int reset_cilia_state(iblb_ctx* c) {
    const size_t nk = (size_t)CILIA_SAMPLES * c->cilia.c_num;
    HIP_TRY(c, hipMemsetAsync(c->cil_samples, 0, 5 * nk * sizeof(float), c->stream));
    HIP_TRY(c, hipMemsetAsync(c->cil_lasts, 0, 2 * nk * sizeof(float), c->stream));
    HIP_TRY(c, hipMemsetAsync(c->cil_bpoints, 0, 5 * (size_t)CILIA_POINTS * c->cilia.c_num * sizeof(float),
                              c->stream));
    return IBLB_OK;
}

int iblb_set_cilia(iblb_ctx* c, const iblb_cilia* k) {
    if (!c) return IBLB_ERR_ARG;
    c->band_valid = false;  // the points now come from the kinematics
    c->sch_n = 0;
    c->sch_cur = -1;
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->ib_state == IB_PENDING) {  // force still owed to the current points
        if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: set cilia between group steps");
        int rc = ensure_force(c);
        if (rc) return rc;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (float* p : {c->cil_samples, c->cil_lasts, c->cil_bpoints})
        if (p) (void)hipFree(p);
    c->cil_samples = c->cil_lasts = c->cil_bpoints = nullptr;
    c->cilia_on = false;
    if (!k || k->c_num <= 0) return IBLB_OK;
    if (k->T <= 0 || !(k->c_space > 0)) return fail(c, IBLB_ERR_ARG, "cilia: need T > 0 and c_space > 0");
    if (CILIA_POINTS * k->c_num > c->max_points)
        return fail(c, IBLB_ERR_ARG, "cilia: max_points must be >= 96 * c_num");
    c->cilia = *k;
    const size_t nk = (size_t)CILIA_SAMPLES * k->c_num;
    HIP_TRY(c, hipMalloc(&c->cil_samples, 5 * nk * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->cil_lasts, 2 * nk * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->cil_bpoints, 5 * (size_t)CILIA_POINTS * k->c_num * sizeof(float)));
    int rc = reset_cilia_state(c);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->cilia_on = true;
    return IBLB_OK;
}

int iblb_get_lagrangian(iblb_ctx* c, float* s, float* u_s, int* epsilon) {
    if (!c) return IBLB_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const size_t ns = (size_t)c->ns;
    if (ns == 0) return IBLB_OK;
    if (s) HIP_TRY(c, hipMemcpy(s, pts_s(c), 2 * ns * sizeof(float), hipMemcpyDeviceToHost));
    if (u_s) HIP_TRY(c, hipMemcpy(u_s, pts_us(c), 2 * ns * sizeof(float), hipMemcpyDeviceToHost));
    if (epsilon) HIP_TRY(c, hipMemcpy(epsilon, pts_eps(c), ns * sizeof(int), hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_step(iblb_ctx* c, int nsteps) {
    if (!c || nsteps < 0) return IBLB_ERR_ARG;
    if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: use iblb_group_step");
    int rc = check_ready(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    for (int s = 0; s < nsteps;) {
        if (c->sch_n > 0 && !c->cilia_on && c->phase == PH_RUN && nsteps - s >= c->sweep_depth &&
            (rc = plan_cycle(c)))
            return rc;
        if (nsteps - s >= c->sweep_depth && band_ready(c)) {
            if ((rc = c->prec == IBLB_PREC_F64 ? band_step<double>(c) : band_step<float>(c))) return rc;
            s += c->sweep_depth;
            continue;
        }
        if (c->sweep_depth >= 3 && nsteps - s >= c->sweep_depth && sweep_ready(c)) {
            if (single_slab(c)) {
                if ((rc = c->prec == IBLB_PREC_F64 ? sweepk_step<double>(c) : sweepk_step<float>(c))) return rc;
                s += c->sweep_depth;
                continue;
            }
            if (rccl_multi(c) && c->ncol >= 2 * c->sweep_depth) {
                if ((rc = c->prec == IBLB_PREC_F64 ? deep_slab_step<double>(c) : deep_slab_step<float>(c))) return rc;
                s += c->sweep_depth;
                continue;
            }
        }
        if (nsteps - s >= 2 && sweep_ready(c)) {
            if ((rc = c->prec == IBLB_PREC_F64 ? sweep_step<double>(c) : sweep_step<float>(c))) return rc;
            s += 2;
            continue;
        }
        if ((rc = step_one(c))) return rc;
        ++s;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return IBLB_OK;
}

int iblb_get_macro(iblb_ctx* c, double* rho, double* u) {
    if (!c) return IBLB_ERR_ARG;
    int rc = prepare_read(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    const long N = (long)c->ncol * c->ny;
    const size_t nb = (size_t)N * sizeof(double);
    DevBuf d;
    HIP_TRY(c, hipMalloc(&d.p, 3 * nb));
    if ((rc = macro_device(c, (double*)d.p, (double*)d.p + N))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (rho) HIP_TRY(c, hipMemcpy(rho, d.p, nb, hipMemcpyDeviceToHost));
    if (u) HIP_TRY(c, hipMemcpy(u, (double*)d.p + N, 2 * nb, hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_get_populations(iblb_ctx* c, double* f) {
    if (!c || !f) return IBLB_ERR_ARG;
    int rc = prepare_read(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    const long N = (long)c->ncol * c->ny;
    DevBuf df;
    HIP_TRY(c, hipMalloc(&df.p, 9 * (size_t)N * sizeof(double)));
    const int raw = c->phase == PH_BOOT;  // f^0 is stored unstreamed
    if (c->prec == IBLB_PREC_F64)
        HIP_TRY(c, launch_pop_out<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), (double*)df.p,
                                          raw, c->stream));
    else
        HIP_TRY(c, launch_pop_out<float>(gptr<float>(c, c->cur), c->L, halo_of<float>(c, c->cur), (double*)df.p, raw,
                                         c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(f, df.p, 9 * (size_t)N * sizeof(double), hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_get_force(iblb_ctx* c, double* force) {
    if (!c || !force) return IBLB_ERR_ARG;
    int rc = prepare_read(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    const long N = (long)c->ncol * c->ny;
    DevBuf d;
    HIP_TRY(c, hipMalloc(&d.p, 2 * (size_t)N * sizeof(double)));
    if (c->phase == PH_BOOT)
        HIP_TRY(c, launch_field_out(c->force0, (double*)d.p, c->L, 2, c->fplane, c->coef.gx, c->coef.gy, c->stream));
    else
        HIP_TRY(c, launch_field_out(c->ib_state == IB_READY ? c->fdense : nullptr, (double*)d.p, c->L, 2, c->fplane,
                                    c->coef.gx, c->coef.gy, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(force, d.p, 2 * (size_t)N * sizeof(double), hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_get_lagrangian_force(iblb_ctx* c, float* F_s) {
    if (!c || !F_s) return IBLB_ERR_ARG;
    int rc = prepare_read(c);
    if (rc) return rc;
    if (c->ns == 0) return IBLB_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    const float* src = c->d_Fs;
    if (rccl_multi(c)) {  // each point's F_s is held by one slab, zeros elsewhere: sum exactly
        NCCL_TRY(c, ncclAllReduce(c->d_Fs, c->d_Fs_sum, 2 * (size_t)c->ns, ncclFloat32, ncclSum, c->comm, c->stream));
        src = c->d_Fs_sum;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(F_s, src, 2 * (size_t)c->ns * sizeof(float), hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_get_flux(iblb_ctx* c, double* Q) {
    if (!c || !Q) return IBLB_ERR_ARG;
    int rc = prepare_read(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    // d_Q[1] = d_Q[0] + q(u^t) of the current (not yet collided) state
    HIP_TRY(c, hipMemcpyAsync(c->d_Q + 1, c->d_Q, sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    const int fc = c->cfg.flux_column - c->x_begin;
    if (c->phase == PH_RUN && fc >= 0 && fc < c->ncol) {
        const double* fd = c->ib_state == IB_READY ? c->fdense : nullptr;
        if (c->prec == IBLB_PREC_F64)
            HIP_TRY(c, launch_flux<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), fd, c->fplane,
                                           c->coef.gx, c->coef.gy, fc, c->cfg.flux_norm, c->d_Q + 1, c->stream));
        else
            HIP_TRY(c, launch_flux<float>(gptr<float>(c, c->cur), c->L, halo_of<float>(c, c->cur), fd, c->fplane,
                                          c->coef.gx, c->coef.gy, fc, c->cfg.flux_norm, c->d_Q + 1, c->stream));
    }
    if (rccl_multi(c))
        NCCL_TRY(c, ncclAllReduce(c->d_Q + 1, c->d_Q + 1, 1, ncclFloat64, ncclSum, c->comm, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(Q, c->d_Q + 1, sizeof(double), hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_get_step(iblb_ctx* c, long long* steps) {
    if (!c || !steps) return IBLB_ERR_ARG;
    *steps = c->t;
    return IBLB_OK;
}

int iblb_set_profiling(iblb_ctx* c, int enabled) {
    if (!c) return IBLB_ERR_ARG;
    c->prof = enabled != 0;
    return IBLB_OK;
}

int iblb_get_timing(iblb_ctx* c, iblb_timing* t, int reset) {
    if (!c || !t) return IBLB_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->comm_stream) HIP_TRY(c, hipStreamSynchronize(c->comm_stream));
    for (auto& r : c->ev_kind) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev_pool[r.idx], c->ev_pool[r.idx + 1]));
        ev_account(c, r, ms);
    }
    c->ev_kind.clear();
    c->ev_used = 0;
    t->steps = c->t;
    t->fused_launches = c->fused_launches;
    t->fused_ms = c->fused_ms;
    t->ib_ms = c->ib_ms;
    t->halo_ms = c->halo_ms;
    t->fused_bytes = 18.0 * (double)c->esize;
    t->cells = (long long)c->ncol * c->ny;
    t->fused_cells = c->fused_cells;
    t->sweep_launches = c->sweep_launches;
    t->sweep_ms = c->sweep_ms;
    t->sweep_cells = c->sweep_cells;
    t->sweepk_launches = c->sweepk_launches;
    t->sweepk_ms = c->sweepk_ms;
    t->sweepk_cells = c->sweepk_cells;
    t->sweepk_depth = c->sweep_depth;
    if (reset) {
        c->fused_ms = c->ib_ms = c->halo_ms = c->sweep_ms = c->sweepk_ms = 0.;
        c->fused_launches = c->fused_cells = c->sweep_launches = c->sweep_cells = 0;
        c->sweepk_launches = c->sweepk_cells = 0;
    }
    return IBLB_OK;
}

int iblb_get_stream(iblb_ctx* c, void** stream) {
    if (!c || !stream) return IBLB_ERR_ARG;
    *stream = (void*)c->stream;
    return IBLB_OK;
}

int iblb_synchronize(iblb_ctx* c) {
    if (!c) return IBLB_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->comm_stream) HIP_TRY(c, hipStreamSynchronize(c->comm_stream));
    return IBLB_OK;
}

// ---- local groups ---------------------------------------------------------------------------
static int sync_all(iblb_ctx** cs, int n) {
    for (int i = 0; i < n; ++i) {
        HIP_TRY(cs[i], hipSetDevice(cs[i]->device));
        HIP_TRY(cs[i], hipStreamSynchronize(cs[i]->stream));
    }
    return IBLB_OK;
}

int iblb_link_local(iblb_ctx** ctxs, int n) {
    if (!ctxs || n < 1) return IBLB_ERR_ARG;
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return IBLB_ERR_ARG;
        iblb_ctx* c = ctxs[i];
        iblb_ctx* nx_ = ctxs[(i + 1) % n];
        if (c->nx != ctxs[0]->nx || c->ny != ctxs[0]->ny || c->prec != ctxs[0]->prec)
            return fail(c, IBLB_ERR_ARG, "local group: slabs differ in lattice size or precision");
        if ((c->x_begin + c->ncol) % c->nx != nx_->x_begin)
            return fail(c, IBLB_ERR_ARG, "local group: slabs must tile the lattice left to right");
    }
    long total = 0;
    for (int i = 0; i < n; ++i) total += ctxs[i]->ncol;
    if (total != ctxs[0]->nx) return fail(ctxs[0], IBLB_ERR_ARG, "local group: slabs do not cover the lattice");
    if (n == 1) return IBLB_OK;  // a single slab is its own periodic neighbour
    for (int i = 0; i < n; ++i) {
        ctxs[i]->transport = TR_LOCAL;
        ctxs[i]->left = ctxs[(i + n - 1) % n];
        ctxs[i]->right = ctxs[(i + 1) % n];
        ctxs[i]->halo_valid = false;
        HIP_TRY(ctxs[i], hipSetDevice(ctxs[i]->device));
        int rc = pack_send(ctxs[i]);  // a restored state has no send buffers yet
        if (rc) return rc;
    }
    return sync_all(ctxs, n);
}

static int group_exchange(iblb_ctx** cs, int n) {
    bool ib = false;  // an owed IB force is evaluated from this halo: carry the IB slots
    for (int i = 0; i < n; ++i) ib |= cs[i]->ib_state == IB_PENDING;
    int rc;
    for (int i = 0; i < n; ++i) {
        if (ib) {
            HIP_TRY(cs[i], hipSetDevice(cs[i]->device));
            if ((rc = pack_ib_any(cs[i], cs[i]->stream))) return rc;
        }
    }
    if ((rc = sync_all(cs, n))) return rc;
    for (int i = 0; i < n; ++i)
        if ((rc = exchange_local(cs[i], ib))) return rc;
    return sync_all(cs, n);
}

static int group_force(iblb_ctx** cs, int n) {
    int rc;
    for (int i = 0; i < n; ++i) {
        if (cs[i]->ib_state != IB_PENDING) continue;
        HIP_TRY(cs[i], hipSetDevice(cs[i]->device));
        if ((rc = ib_slab_any(cs[i]))) return rc;
    }
    return sync_all(cs, n);
}

int iblb_group_step(iblb_ctx** cs, int n, int nsteps) {
    if (!cs || n < 1 || nsteps < 0) return IBLB_ERR_ARG;
    if (n == 1) return iblb_step(cs[0], nsteps);
    for (int i = 0; i < n; ++i) {
        if (!cs[i] || cs[i]->transport != TR_LOCAL) return IBLB_ERR_ARG;
        if (cs[i]->phase == PH_EMPTY) return fail(cs[i], IBLB_ERR_STATE, "no state: call iblb_set_state first");
        if (cs[i]->phase != cs[0]->phase || cs[i]->t != cs[0]->t || cs[i]->ns != cs[0]->ns)
            return fail(cs[i], IBLB_ERR_STATE, "local group: slabs out of step");
    }
    int rc;
    for (int s = 0; s < nsteps; ++s) {
        if (cs[0]->phase == PH_RUN) {
            const bool ib = cs[0]->ib_state == IB_PENDING;
            if ((!cs[0]->halo_valid || (ib && !cs[0]->halo_ib)) && (rc = group_exchange(cs, n))) return rc;
            if ((rc = group_force(cs, n))) return rc;
        }
        for (int i = 0; i < n; ++i) {
            if (!cs[i]->cilia_on) continue;
            HIP_TRY(cs[i], hipSetDevice(cs[i]->device));
            if ((rc = run_cilia(cs[i]))) return rc;
        }
        for (int i = 0; i < n; ++i) {
            HIP_TRY(cs[i], hipSetDevice(cs[i]->device));
            if ((rc = advance(cs[i]))) return rc;
        }
    }
    // leave the group readable: halos of the new state and its force^t
    if ((rc = group_exchange(cs, n))) return rc;
    if ((rc = group_force(cs, n))) return rc;
    for (int i = 0; i < n; ++i)
        if (cs[i]->phase == PH_RUN && cs[i]->t >= 1 && cs[i]->rho0) free_boot(cs[i]);
    return sync_all(cs, n);
}

// ---- RCCL groups ------------------------------------------------------------------------------
int iblb_rccl_unique_id(char id[IBLB_UNIQUE_ID_BYTES]) {
    if (!id) return IBLB_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == IBLB_UNIQUE_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return fail(nullptr, IBLB_ERR_COMM, "ncclGetUniqueId failed");
    std::memcpy(id, &u, sizeof(u));
    return IBLB_OK;
}

int iblb_attach_rccl(iblb_ctx* c, const char id[IBLB_UNIQUE_ID_BYTES], int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return IBLB_ERR_ARG;
    c->deep_chain = false;  // the state is rewritten: no deep cycle chain across this
    if (c->transport != TR_NONE) return fail(c, IBLB_ERR_STATE, "context already linked");
    HIP_TRY(c, hipSetDevice(c->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    NCCL_TRY(c, ncclCommInitRank(&c->comm, nranks, u, rank));
    c->nranks = nranks;
    c->rank = rank;
    c->transport = TR_RCCL;
    // IBLB_RCCL_SELF=1 with one rank: the slab exchanges its halo with itself through RCCL, so
    // the multi-slab schedule (comm stream, overlap, node all-reduce) runs on one GPU
    c->self_ring = nranks == 1 && env_long("IBLB_RCCL_SELF", 0) != 0;
    if (nranks > 1) {
        // the slabs must tile the lattice in rank order: check (x_begin, ncol) of all ranks
        DevBuf d;
        HIP_TRY(c, hipMalloc(&d.p, 2 * sizeof(int) * (size_t)nranks));
        int mine[2] = {c->x_begin, c->ncol};
        HIP_TRY(c, hipMemcpy((int*)d.p + 2 * rank, mine, sizeof(mine), hipMemcpyHostToDevice));
        NCCL_TRY(c, ncclAllGather((int*)d.p + 2 * rank, d.p, 2, ncclInt32, c->comm, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        std::vector<int> all(2 * (size_t)nranks);
        HIP_TRY(c, hipMemcpy(all.data(), d.p, all.size() * sizeof(int), hipMemcpyDeviceToHost));
        long total = 0;
        for (int r = 0; r < nranks; ++r) {
            total += all[2 * r + 1];
            const int nxt = (r + 1) % nranks;
            if ((all[2 * r] + all[2 * r + 1]) % c->nx != all[2 * nxt])
                return fail(c, IBLB_ERR_ARG, "RCCL group: slabs must tile the lattice in rank order");
        }
        if (total != c->nx) return fail(c, IBLB_ERR_ARG, "RCCL group: slabs do not cover the lattice");
        c->slab_begin.resize(nranks);
        c->slab_count.resize(nranks);
        for (int r = 0; r < nranks; ++r) {
            c->slab_begin[r] = all[2 * r];
            c->slab_count[r] = all[2 * r + 1];
        }
    } else {
        if (c->self_ring && c->ncol != c->nx) return fail(c, IBLB_ERR_ARG, "IBLB_RCCL_SELF needs the whole lattice");
        c->slab_begin.assign(1, c->x_begin);
        c->slab_count.assign(1, c->ncol);
    }
    if (rccl_multi(c)) {
        // The halo's RCCL kernels run beside the interior collide, which fills every CU: give
        // the comm stream the highest priority (its workgroups go first as CUs free up) and,
        // optionally, keep IBLB_RESERVE_CUS compute units free of the collide for them.
        // 8 reserved CUs: 512 x 4096 f64 slab step 0.070 ms vs 0.165 ms without (self-ring
        // rehearsal, profiles/r01e_gap_probe.txt); 4 or 16 are within 1 %
        hipDeviceProp_t prop;
        HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
        c->ncu = prop.multiProcessorCount;
        long reserve = env_long("IBLB_RESERVE_CUS", 8);
        if (c->sweep_depth >= 3 && env_long("IBLB_RESERVE_CUS", -1) < 0) {
            // deep slabs: enough CUs for every wave of the two boundary sweeps to be resident
            // at once (they walk K-1 columns more than they write and sit on the critical path of
            // the comm stream: exchange -> boundary -> pack)
            int nch = 0;
            const int wpc = c->prec == IBLB_PREC_F64
                                ? sweepk_geometry<double>(c->sweep_depth, c->deep_bnd_vs, c->deep_variant, true, c->ny, &nch)
                                : sweepk_geometry<float>(c->sweep_depth, c->deep_bnd_vs, c->deep_variant, true, c->ny, &nch);
            // rounded up to multiples of ncu / 8 (the top mask bits take the same number of CUs
            // from every XCD, profiles/r02n_xcc_probe.txt); 32 measured best (self ring, deep
            // slab 512 / 1024 / 2048 x 4096: 0.0376 / 0.0564 / 0.0953 ms/iteration with 32 CUs,
            // 0.046 / 0.080 / 0.148 with 16, 0.049 / 0.087 / 0.164 with 40;
            // profiles/r01e5_gap_probe_reserve.txt)
            if (wpc > 0) {
                const long need = std::max(8L, (long)((2 * nch + wpc - 1) / wpc));
                const long xcd = std::max(1, c->ncu / 8);
                reserve = std::min((long)c->ncu / 2, (need + xcd - 1) / xcd * xcd);
            }
        }
        if (reserve > 0) {
            const int ncu = c->ncu;
            if (reserve >= ncu) return fail(c, IBLB_ERR_ARG, "IBLB_RESERVE_CUS exceeds the compute units");
            // Which CUs: the top mask bits.  Bit i is a CU of XCD i % 8 and the dispatcher deals
            // workgroups round-robin over all eight XCDs whatever the mask (an XCD left without
            // any bit runs on all its CUs), so the top 32 bits are four CUs of every XCD
            // (profiles/r02n_xcc_probe.txt).  IBLB_RESERVE_LAYOUT=1 picks bits 31, 63, ..., i.e.
            // all of XCD 7, which then falls back to unmasked: measured slower (0.0486 vs
            // 0.0376 ms/iteration with 32, profiles/r01e4_*).
            const bool xcd_major = env_long("IBLB_RESERVE_LAYOUT", 0) == 1 && ncu % 8 == 0;
            if (xcd_major) reserve = (reserve + 7) / 8 * 8;
            if (reserve >= ncu) return fail(c, IBLB_ERR_ARG, "IBLB_RESERVE_CUS exceeds the compute units");
            std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
            for (int i = 0; i < ncu; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
            const int per_xcd = ncu / 8;
            for (long k = 0; k < reserve; ++k) {
                const long i = xcd_major ? (k % 8) * per_xcd + (per_xcd - 1 - k / 8) : ncu - 1 - k;
                mask[(size_t)i / 32] &= ~(1u << (i % 32));
            }
            hipStream_t masked = nullptr;
            HIP_TRY(c, hipExtStreamCreateWithCUMask(&masked, (uint32_t)mask.size(), mask.data()));
            c->reserved_cus = (int)reserve;
            c->comp_mask = mask;
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            (void)hipStreamDestroy(c->stream);
            c->stream = masked;
        }
        int prio_lo = 0, prio_hi = 0;
        HIP_TRY(c, hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
        const int prio = env_long("IBLB_COMM_PRIORITY", 1) != 0 ? prio_hi : prio_lo;
        if (c->reserved_cus > 0 && env_long("IBLB_COMM_MASK", 1) != 0) {
            // the comm stream confined to the reserved CUs: a boundary sweep dispatched before the
            // interior of the same cycle must not take CUs the interior's round of waves needs
            std::vector<uint32_t> m(c->comp_mask.size(), 0u);
            for (int i = 0; i < c->ncu; ++i)
                if (!(c->comp_mask[(size_t)i / 32] >> (i % 32) & 1u)) m[(size_t)i / 32] |= 1u << (i % 32);
            HIP_TRY(c, hipExtStreamCreateWithCUMask(&c->comm_stream, (uint32_t)m.size(), m.data()));
        } else {
            HIP_TRY(c, hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, prio));
        }
        // cross-stream ordering events (producer and consumer on this device): IBLB_EVENT_FENCE
        // 0 = HIP's default system-scope release / acquire, 1 = hipEventDisableSystemFence
        // (default: 512 x 4096 self ring 0.0394 vs 0.0420 ms/iteration, 1024 0.0682 vs 0.0705,
        // profiles/r01u_gap_probe_event_fence.txt), 2 = hipEventReleaseToDevice
        const long ef = env_long("IBLB_EVENT_FENCE", 1);
        const unsigned evf = hipEventDisableTiming |
                             (ef == 1 ? hipEventDisableSystemFence : (ef == 2 ? hipEventReleaseToDevice : 0u));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_bnd, evf));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_int, evf));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_pre, evf));
        c->sweep_order = (int)env_long("IBLB_SWEEP_ORDER", 0);
        c->deep_order = (int)env_long("IBLB_DEEP_ORDER", 1);

        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));  // send buffers of the current state
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        c->overlap = env_long("IBLB_OVERLAP", 1) != 0;
    }
    c->halo_valid = false;
    int rc = pack_send(c);  // a restored state has no send buffers yet
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return IBLB_OK;
}

// ---- output gather (RCCL group) -----------------------------------------------------------
int iblb_gather_macro(iblb_ctx* c, int root, double* rho, double* u) {
    if (!c) return IBLB_ERR_ARG;
    if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: gather the slabs' iblb_get_macro");
    if (!rccl_multi(c)) return iblb_get_macro(c, rho, u);
    if (root < 0 || root >= c->nranks) return fail(c, IBLB_ERR_ARG, "root rank out of range");
    int rc = prepare_read(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    const long N = (long)c->ncol * c->ny;
    DevBuf mine, all;
    HIP_TRY(c, hipMalloc(&mine.p, 3 * (size_t)N * sizeof(double)));
    if ((rc = macro_device(c, (double*)mine.p, (double*)mine.p + N))) return rc;
    const bool is_root = c->rank == root;
    const size_t total = 3 * (size_t)c->nx * c->ny;
    if (is_root) HIP_TRY(c, hipMalloc(&all.p, total * sizeof(double)));
    // rank r's [rho | u] block lands at 3*ny*x_begin_r in rank order
    NCCL_TRY(c, ncclGroupStart());
    if (is_root) {
        for (int r = 0; r < c->nranks; ++r) {
            double* dst = (double*)all.p + 3L * c->ny * c->slab_begin[r];
            const size_t n = 3 * (size_t)c->ny * c->slab_count[r];
            if (r == root)
                HIP_TRY(c, hipMemcpyAsync(dst, mine.p, n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
            else
                NCCL_TRY(c, ncclRecv(dst, n, ncclFloat64, r, c->comm, c->stream));
        }
    } else {
        NCCL_TRY(c, ncclSend(mine.p, 3 * (size_t)N, ncclFloat64, root, c->comm, c->stream));
    }
    NCCL_TRY(c, ncclGroupEnd());
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (!is_root || (!rho && !u)) return IBLB_OK;
    std::vector<double> h(total);
    HIP_TRY(c, hipMemcpy(h.data(), all.p, total * sizeof(double), hipMemcpyDeviceToHost));
    const long nx = c->nx, ny = c->ny, G = nx * ny;
    for (int r = 0; r < c->nranks; ++r) {
        const long xb = c->slab_begin[r], nc = c->slab_count[r], n = nc * ny;
        const double* blk = h.data() + 3 * ny * xb;
        for (long y = 0; y < ny; ++y)
            for (long xc = 0; xc < nc; ++xc) {
                const long j = y * nc + xc, g = y * nx + xb + xc;
                if (rho) rho[g] = blk[j];
                if (u) {
                    u[g] = blk[n + j];
                    u[G + g] = blk[2 * n + j];
                }
            }
    }
    return IBLB_OK;
}

// ---- checkpoint / restart ---------------------------------------------------------------------
// File: 8-byte magic, 12 int64 fields, 6 doubles, then the stored populations g (plane i, column
// xc, rows y; storage precision, no padding), the Lagrangian points and the cilia buffers.
namespace {
const char CKPT_MAGIC[8] = {'I', 'B', 'L', 'B', 'C', 'K', '0', '1'};
enum { CK_VERSION, CK_NX, CK_NY, CK_XB, CK_NCOL, CK_PREC, CK_T, CK_NS, CK_CILIA, CK_CNUM, CK_CT, CK_CPSTEP, CK_NI };
enum { CK_Q, CK_CSPACE, CK_TAU, CK_TAU2, CK_GX, CK_GY, CK_ND };

struct File {
    FILE* f = nullptr;
    ~File() { if (f) std::fclose(f); }
};

int ck_io(iblb_ctx* c, bool ok) { return ok ? IBLB_OK : fail(c, IBLB_ERR_ARG, "checkpoint file truncated or unwritable"); }

// device <-> file through a host bounce buffer
int ck_dev(iblb_ctx* c, File& fl, bool save, void* dev, size_t bytes) {
    if (bytes == 0) return IBLB_OK;
    std::vector<char> h(bytes);
    if (save) {
        HIP_TRY(c, hipMemcpy(h.data(), dev, bytes, hipMemcpyDeviceToHost));
        return ck_io(c, std::fwrite(h.data(), 1, bytes, fl.f) == bytes);
    }
    if (std::fread(h.data(), 1, bytes, fl.f) != bytes) return ck_io(c, false);
    HIP_TRY(c, hipMemcpy(dev, h.data(), bytes, hipMemcpyHostToDevice));
    return IBLB_OK;
}

int ck_pops(iblb_ctx* c, File& fl, bool save) {
    const size_t w = (size_t)c->ny * c->esize, pitch = (size_t)c->L.col * c->esize;
    std::vector<char> h(w * c->ncol);
    for (int i = 0; i < 9; ++i) {
        char* plane = (char*)c->g[c->cur] + (size_t)i * c->L.plane * c->esize;
        if (save) {
            HIP_TRY(c, hipMemcpy2D(h.data(), w, plane, pitch, w, c->ncol, hipMemcpyDeviceToHost));
            if (std::fwrite(h.data(), 1, h.size(), fl.f) != h.size()) return ck_io(c, false);
        } else {
            if (std::fread(h.data(), 1, h.size(), fl.f) != h.size()) return ck_io(c, false);
            HIP_TRY(c, hipMemcpy2D(plane, pitch, h.data(), w, w, c->ncol, hipMemcpyHostToDevice));
        }
    }
    return IBLB_OK;
}

}  // namespace

int iblb_save_checkpoint(iblb_ctx* c, const char* path) {
    if (!c || !path) return IBLB_ERR_ARG;
    if (c->phase != PH_RUN) return fail(c, IBLB_ERR_STATE, "checkpoint needs a state advanced by at least one step");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->comm_stream) HIP_TRY(c, hipStreamSynchronize(c->comm_stream));
    File fl;
    const std::string tmp = std::string(path) + ".tmp";
    fl.f = std::fopen(tmp.c_str(), "wb");
    if (!fl.f) return fail(c, IBLB_ERR_ARG, std::string("cannot open ") + tmp + " for writing");
    double Q = 0.;
    HIP_TRY(c, hipMemcpy(&Q, c->d_Q, sizeof(double), hipMemcpyDeviceToHost));
    long long iv[CK_NI] = {1, c->nx, c->ny, c->x_begin, c->ncol, c->prec, c->t, c->ns, c->cilia_on ? 1 : 0,
                           c->cilia.c_num, c->cilia.T, c->cilia.p_step};
    double dv[CK_ND] = {Q, c->cilia.c_space, c->cfg.tau, c->cfg.tau2, c->coef.gx, c->coef.gy};
    int rc = ck_io(c, std::fwrite(CKPT_MAGIC, 1, 8, fl.f) == 8 && std::fwrite(iv, sizeof(iv), 1, fl.f) == 1 &&
                          std::fwrite(dv, sizeof(dv), 1, fl.f) == 1);
    if (rc || (rc = ck_pops(c, fl, true))) return rc;
    const size_t ns = (size_t)c->ns;
    // (under a schedule: the entry in use; the restart continues with those points)
    if ((rc = ck_dev(c, fl, true, (void*)pts_s(c), 2 * ns * sizeof(float))) ||
        (rc = ck_dev(c, fl, true, (void*)pts_us(c), 2 * ns * sizeof(float))) ||
        (rc = ck_dev(c, fl, true, (void*)pts_eps(c), ns * sizeof(int))))
        return rc;
    if (c->cilia_on) {
        const size_t nk = (size_t)CILIA_SAMPLES * c->cilia.c_num;
        if ((rc = ck_dev(c, fl, true, c->cil_samples, 5 * nk * sizeof(float))) ||
            (rc = ck_dev(c, fl, true, c->cil_lasts, 2 * nk * sizeof(float))) ||
            (rc = ck_dev(c, fl, true, c->cil_bpoints, 5 * (size_t)CILIA_POINTS * c->cilia.c_num * sizeof(float))))
            return rc;
    }
    const bool ok = std::fflush(fl.f) == 0;
    std::fclose(fl.f);
    fl.f = nullptr;
    if (!ok || std::rename(tmp.c_str(), path) != 0) return fail(c, IBLB_ERR_ARG, std::string("cannot write ") + path);
    return IBLB_OK;
}

int iblb_load_checkpoint(iblb_ctx* c, const char* path) {
    if (!c || !path) return IBLB_ERR_ARG;
    c->deep_chain = false;  // the state is rewritten: no deep cycle chain across this
    if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: restore the slabs before linking");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    File fl;
    fl.f = std::fopen(path, "rb");
    if (!fl.f) return fail(c, IBLB_ERR_ARG, std::string("cannot open ") + path);
    char magic[8];
    long long iv[CK_NI];
    double dv[CK_ND];
    if (std::fread(magic, 1, 8, fl.f) != 8 || std::memcmp(magic, CKPT_MAGIC, 8) != 0)
        return fail(c, IBLB_ERR_ARG, "not an iblb checkpoint");
    if (std::fread(iv, sizeof(iv), 1, fl.f) != 1 || std::fread(dv, sizeof(dv), 1, fl.f) != 1) return ck_io(c, false);
    if (iv[CK_VERSION] != 1) return fail(c, IBLB_ERR_ARG, "unsupported checkpoint version");
    if (iv[CK_NX] != c->nx || iv[CK_NY] != c->ny || iv[CK_XB] != c->x_begin || iv[CK_NCOL] != c->ncol ||
        iv[CK_PREC] != c->prec)
        return fail(c, IBLB_ERR_ARG, "checkpoint lattice/slab/precision differs from the context");
    if (dv[CK_TAU] != c->cfg.tau || dv[CK_TAU2] != c->cfg.tau2 || dv[CK_GX] != c->coef.gx || dv[CK_GY] != c->coef.gy)
        return fail(c, IBLB_ERR_ARG, "checkpoint relaxation times / body force differ from the context");
    if (iv[CK_NS] > c->max_points) return fail(c, IBLB_ERR_ARG, "checkpoint holds more points than max_points");
    int rc;
    // cilia configuration first (allocates its buffers), then every array
    if (iv[CK_CILIA]) {
        iblb_cilia k{(int)iv[CK_CNUM], dv[CK_CSPACE], (int)iv[CK_CT], (int)iv[CK_CPSTEP]};
        c->ib_state = IB_NONE;
        if ((rc = iblb_set_cilia(c, &k))) return rc;
    } else if (c->cilia_on) {
        c->ib_state = IB_NONE;
        if ((rc = iblb_set_cilia(c, nullptr))) return rc;
    }
    if ((rc = ck_pops(c, fl, false))) return rc;
    const size_t ns = (size_t)iv[CK_NS];
    if ((rc = ck_dev(c, fl, false, c->d_s, 2 * ns * sizeof(float))) ||
        (rc = ck_dev(c, fl, false, c->d_us, 2 * ns * sizeof(float))) ||
        (rc = ck_dev(c, fl, false, c->d_eps, ns * sizeof(int))))
        return rc;
    if (c->cilia_on) {
        const size_t nk = (size_t)CILIA_SAMPLES * c->cilia.c_num;
        if ((rc = ck_dev(c, fl, false, c->cil_samples, 5 * nk * sizeof(float))) ||
            (rc = ck_dev(c, fl, false, c->cil_lasts, 2 * nk * sizeof(float))) ||
            (rc = ck_dev(c, fl, false, c->cil_bpoints, 5 * (size_t)CILIA_POINTS * c->cilia.c_num * sizeof(float))))
            return rc;
    }
    free_boot(c);
    double q[4] = {dv[CK_Q], 0., 0., 0.};
    HIP_TRY(c, hipMemcpy(c->d_Q, q, sizeof(q), hipMemcpyHostToDevice));
    if (c->fdense) {
        HIP_TRY(c, hipMemsetAsync(c->fdense, 0, 2 * (size_t)c->fplane * sizeof(double), c->stream));
        HIP_TRY(c, hipMemsetAsync(c->flags, 0, (size_t)c->ncol * c->nch, c->stream));
    }
    c->ns = (int)ns;
    c->sch_n = 0;  // the restored points are static
    c->sch_cur = -1;
    c->band_sticky = false;
    c->band_valid = false;
    if (ns > 0 && !c->cilia_on) {  // the band plan of the restored points
        std::vector<float> hs(2 * ns);
        HIP_TRY(c, hipMemcpy(hs.data(), c->d_s, hs.size() * sizeof(float), hipMemcpyDeviceToHost));
        if ((rc = plan_bands(c, x_coords((int)ns, hs.data())))) return rc;
    }
    c->t = iv[CK_T];
    c->phase = PH_RUN;
    c->halo_valid = false;
    c->ib_state = ib_active(c) ? IB_PENDING : IB_NONE;  // force^t is re-evaluated from g and the points
    if ((rc = pack_send(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return IBLB_OK;
}

}  // extern "C"
