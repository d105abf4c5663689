// ctx_step.hip — time stepping of a context (ctx.h): the ghost-column halo exchange, the one-step,
// two-step and deep (K-iteration) schedules of a lone slab and of a slab of a group, iblb_step,
// local groups, RCCL groups and the output gather.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ctx.h"

namespace iblbh {

// ---- halo -------------------------------------------------------------------------------------
// RCCL calls of one communicator must execute in issue order on every rank: a call on another
// stream than the previous one waits for it.
int rccl_order(iblb_ctx* c, hipStream_t st) {
    if (c->rccl_last && c->rccl_last != st) {
        HIP_TRY(c, hipEventRecord(c->ev_rccl, c->rccl_last));
        HIP_TRY(c, hipStreamWaitEvent(st, c->ev_rccl, 0));
    }
    c->rccl_last = st;
    return IBLB_OK;
}

// Compute stream after the comm-stream work of the last step (boundary columns, exchanges).
int join_comm(iblb_ctx* c) {
    if (c->comm_stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_bnd, 0));
    return IBLB_OK;
}

// Ghost columns of the current state from the neighbours: the d columns next to each edge, one
// contiguous block of whole columns each way (ncclSend of my columns [0, d) to the left
// neighbour's columns [ncol, ncol+d), of [ncol-d, ncol) to the right neighbour's [-d, 0)).
// With two ranks both neighbours are the same peer: sends and receives pair up in issue order
// (my first send lands in its first receive, its left ghosts).
int exchange(iblb_ctx* c, hipStream_t st, int d) {
    if (d > c->gc || d > c->ncol) return fail(c, IBLB_ERR_ARG, "halo deeper than the ghost columns or the slab");
    int rc = rccl_order(c, st);
    if (rc) return rc;
    if (c->hold_x >= 0 && c->n_exch == c->hold_x) {  // IBLB_TEST_HOLD: this exchange starts late
        if ((rc = hold_release(c))) return rc;
        __atomic_store_n(c->hold_word, 0u, __ATOMIC_RELEASE);
        const double bound_s = c->hold_ms * 1e-3 + 60.;
        HIP_TRY(c, launch_test_hold(c->hold_word, (unsigned long long)(bound_s * c->clock_hz), st));
        std::fprintf(stderr, "iblb: IBLB_TEST_HOLD: exchange %lld (t = %lld) held for %d ms\n", c->n_exch, c->t, c->hold_ms);
        c->hold_thread = std::thread([w = c->hold_word, ms = c->hold_ms] {
            std::this_thread::sleep_for(std::chrono::milliseconds(ms));
            __atomic_store_n(w, 1u, __ATOMIC_RELEASE);
        });
    }
    ++c->n_exch;
    size_t ev = 0;
    if ((rc = ev_begin(c, &ev, st))) return rc;
    char* g = (char*)c->g[c->cur];
    const size_t cb = (size_t)c->L.col * c->esize;
    const size_t n = (size_t)d * c->L.col;
    const ncclDataType_t dt = is_f64(c) ? ncclFloat64 : ncclFloat32;
    const int lr = (c->rank + c->nranks - 1) % c->nranks, rr = (c->rank + 1) % c->nranks;
    NCCL_TRY(c, ncclGroupStart());
    NCCL_TRY(c, ncclSend(g + (size_t)(c->ncol - d) * cb, n, dt, rr, c->comm, st));
    NCCL_TRY(c, ncclSend(g, n, dt, lr, c->comm, st));
    NCCL_TRY(c, ncclRecv(g - (size_t)d * cb, n, dt, lr, c->comm, st));
    NCCL_TRY(c, ncclRecv(g + (size_t)c->ncol * cb, n, dt, rr, c->comm, st));
    NCCL_TRY(c, ncclGroupEnd());
    c->ghost = d;
    return ev_end(c, ev, EV_HALO, 0, st);
}

// A lone slab's ghost columns of buffer `which` as periodic copies of its edge columns.
int fill_ghosts_periodic(iblb_ctx* c, int which, int d, hipStream_t st) {
    if (d > c->gc || d > c->ncol) return fail(c, IBLB_ERR_ARG, "ghost depth exceeds the ghost columns or the slab");
    char* g = (char*)c->g[which];
    const size_t cb = (size_t)c->L.col * c->esize;
    HIP_TRY(c, hipMemcpyAsync(g - (size_t)d * cb, g + (size_t)(c->ncol - d) * cb, (size_t)d * cb,
                              hipMemcpyDeviceToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(g + (size_t)c->ncol * cb, g, (size_t)d * cb, hipMemcpyDeviceToDevice, st));
    return IBLB_OK;
}

// the comm stream is about to send the d edge columns of the current state: follow the compute
// work of the last step unless the comm stream wrote them itself
static int int_event(iblb_ctx* c);
static int comm_ready(iblb_ctx* c, int d) {
    if (d > c->bnd_w) {
        int rc = int_event(c);
        if (rc) return rc;
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_int, 0));
    }
    return IBLB_OK;
}

// Ghosts of the current state for a context that is alone or in an RCCL group (local groups:
// group code): one column, three when an owed IB force is evaluated from them (nodes reach two
// columns beyond the slab, their pulls three).
int ensure_halo(iblb_ctx* c) {
    if (single_slab(c)) return IBLB_OK;
    const int need = c->ib_state == IB_PENDING ? 3 : 1;
    if (c->ghost >= need) return IBLB_OK;
    if (c->transport != TR_RCCL)
        return fail(c, IBLB_ERR_STATE, "slab halo not available: link the slabs (iblb_link_local / iblb_attach_rccl)");
    int rc = join_comm(c);  // the edge columns may have been written on the comm stream
    if (rc) return rc;
    return exchange(c, c->stream, need);
}

// ---- immersed boundary ------------------------------------------------------------------------
int ib_ghost(iblb_ctx* c, const void* g, int gc, int clo, int chi, const float* s, const float* us, const int* eps,
             int part, hipStream_t st, unsigned* sig, unsigned sig_val, int wlo, int whi) {
    IbGhost G{c->nx, c->x_begin, gc, clo, chi, part, sig, sig_val, wlo, whi};
    if (is_f64(c))
        HIP_TRY(c, launch_ib_ghost<double>((const double*)g, c->L, G, c->ns, s, us, eps, c->d_Fs, c->fdense, c->fplane,
                                           c->flags, c->nch, 64 * c->V, st));
    else
        HIP_TRY(c, launch_ib_ghost<float>((const float*)g, c->L, G, c->ns, s, us, eps, c->d_Fs, c->fdense, c->fplane,
                                          c->flags, c->nch, 64 * c->V, st));
    return IBLB_OK;
}

// force^t of the current state.  The dense force and its flags are clean here: the collide that
// consumed the previous force cleared both.  A lone slab: every point in one launch
// (ib_point_kernel); a slab: the points spreading into its columns, from three ghost columns.
int ensure_force(iblb_ctx* c) {
    if (c->ib_state != IB_PENDING) return IBLB_OK;
    if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: advance with iblb_group_step");
    int rc = ensure_halo(c);
    if (rc) return rc;
    size_t ev = 0;
    if ((rc = ev_begin(c, &ev))) return rc;
    if (single_slab(c)) {
        if (is_f64(c))
            HIP_TRY(c, launch_ib_point<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), c->nx, c->ns,
                                               pts_s(c), pts_us(c), pts_eps(c), c->d_Fs, c->fdense, c->fplane, c->flags,
                                               c->nch, 64 * c->V, c->stream));
        else
            HIP_TRY(c, launch_ib_point<float>(gptr<float>(c, c->cur), c->L, halo_of<float>(c, c->cur), c->nx, c->ns,
                                              pts_s(c), pts_us(c), pts_eps(c), c->d_Fs, c->fdense, c->fplane, c->flags,
                                              c->nch, 64 * c->V, c->stream));
    } else {
        if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
        if ((rc = ib_ghost(c, c->g[c->cur], c->ghost, 0, c->ncol, pts_s(c), pts_us(c), pts_eps(c), 0, c->stream)))
            return rc;
    }
    c->ib_state = IB_READY;
    return ev_end(c, ev, EV_IB);
}

// ---- one iteration ----------------------------------------------------------------------------
template <typename T>
static int launch_fused_step(iblb_ctx* c, int col_begin, int ncols, int col_step = 1, bool timed = true,
                             hipStream_t st = nullptr) {
    FusedArgs<T> a{};
    a.src = gptr<T>(c, c->cur);
    a.dst = gptr<T>(c, 1 - c->cur);
    a.L = c->L;
    a.H = halo_of<T>(c, c->cur);
    a.col_begin = col_begin;
    a.col_step = col_step;
    a.ncols = ncols;
    a.cols = nullptr;
    a.nch = c->nch;
    a.flags = c->ib_state == IB_READY ? c->flags : nullptr;
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
    int rc = timed ? ev_begin(c, &ev, st) : IBLB_OK;
    if (rc) return rc;
    HIP_TRY(c, launch_fused<T>(a, st ? st : c->stream));
    return timed ? ev_end(c, ev, EV_FUSED, (long long)ncols * c->ny, st) : IBLB_OK;
}

static void after_step(iblb_ctx* c) {
    c->cur = 1 - c->cur;
    c->t++;
    c->ghost = 0;
    c->ib_state = ib_active(c) ? IB_PENDING : IB_NONE;
}

// the compute stream wrote the whole state: the comm stream follows it
static int comm_follows(iblb_ctx* c) {
    if (!rccl_multi(c)) return IBLB_OK;
    HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
    HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_bnd, 0));
    c->int_unrec = false;
    c->bnd_w = INT_MAX;
    return IBLB_OK;
}

// One reference iteration for a context whose ghosts (if any) and force^t are in place.
static int advance(iblb_ctx* c) {
    int rc;
    if (c->phase == PH_BOOT) {
        if (is_f64(c))
            HIP_TRY(c, launch_boot<double>(gptr<double>(c, c->cur), gptr<double>(c, 1 - c->cur), c->L, c->rho0, c->u0,
                                           c->force0, c->fplane, c->coef, c->kc, c->stream));
        else
            HIP_TRY(c, launch_boot<float>(gptr<float>(c, c->cur), gptr<float>(c, 1 - c->cur), c->L, c->rho0, c->u0,
                                          c->force0, c->fplane, c->coef, c->kc, c->stream));
        c->phase = PH_RUN;
    } else {
        rc = is_f64(c) ? launch_fused_step<double>(c, 0, c->ncol) : launch_fused_step<float>(c, 0, c->ncol);
        if (rc) return rc;
    }
    if ((rc = comm_follows(c))) return rc;
    after_step(c);
    return IBLB_OK;
}

// RCCL slab, no IB force owed.  Step t on two streams:
//   comm:    [after the compute work of t-1 if it wrote the edge columns] exchange(t, 1 column)
//            -> wait int(t-1) -> boundary columns 0, ncol-1 (t) -> ev_bnd
//   compute: (join_comm: boundary(t-1)) -> interior columns [1, ncol-1)(t) -> ev_int
// The interior needs nothing from the exchange, so the halo and the two boundary columns run
// beside it.  boundary(t) waits for interior(t-1): it overwrites columns of the buffer
// interior(t-1) read.
template <typename T>
static int overlapped_step(iblb_ctx* c) {
    int rc = comm_ready(c, 1);
    if (rc || (rc = exchange(c, c->comm_stream, 1)) || (rc = int_event(c))) return rc;
    HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_int, 0));
    if ((rc = launch_fused_step<T>(c, 0, 2, c->ncol - 1, false, c->comm_stream))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_bnd, c->comm_stream));
    if ((rc = launch_fused_step<T>(c, 1, c->ncol - 2))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
    c->bnd_w = 1;
    after_step(c);
    return IBLB_OK;
}

// RCCL slab with an IB force owed (force^t of the points of iteration t-1), step t on two streams:
//   compute: (join_comm) -> IB of the inner points -> ev_pre -> interior columns [3, ncol-3)(t) -> ev_int
//   comm:    wait int(t-1) -> exchange(t, 3 columns) -> IB of the edge points -> wait ev_pre ->
//            boundary columns [0, 3) and [ncol-3, ncol)(t) -> ev_bnd
// Inner points (2 <= x0 - x_begin <= ncol-3: nodes and pulls inside the slab) need no ghosts and
// spread into columns [1, ncol-2]; edge points need the ghosts and spread into columns <= 2 and
// >= ncol-3 only, so the interior collide waits for neither the exchange nor the edge IB.
// boundary(t) waits for the inner IB (its columns 1, 2 / ncol-3, ncol-2 may hold inner forces).
// next: the schedule entry the iteration's points switch to after the owed force (-1: unchanged).
template <typename T>
static int ib_overlapped_step(iblb_ctx* c, int next) {
    hipStream_t bs = c->comm_stream;
    int rc = ib_ghost(c, c->g[c->cur], 0, 0, c->ncol, pts_s(c), pts_us(c), pts_eps(c), 1, c->stream);
    if (rc) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_pre, c->stream));
    if ((rc = int_event(c))) return rc;
    HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_int, 0));
    if ((rc = exchange(c, bs, 3))) return rc;
    if ((rc = ib_ghost(c, c->g[c->cur], 3, 0, c->ncol, pts_s(c), pts_us(c), pts_eps(c), 2, bs))) return rc;
    c->ib_state = IB_READY;
    if (next >= 0) sched_use(c, next);
    HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_pre, 0));
    if ((rc = launch_fused_step<T>(c, 0, 3, 1, false, bs))) return rc;
    if ((rc = launch_fused_step<T>(c, c->ncol - 3, 3, 1, false, bs))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
    if ((rc = launch_fused_step<T>(c, 3, c->ncol - 6))) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
    c->bnd_w = 3;
    after_step(c);
    return IBLB_OK;
}

// ---- several iterations per launch --------------------------------------------------------------
template <typename T>
Sweep2Args<T> sweep_args(iblb_ctx* c, int col_begin, int col_step, int col_end, int nsweep, int W) {
    Sweep2Args<T> a{};
    a.src = gptr<T>(c, c->cur);
    a.dst = gptr<T>(c, 1 - c->cur);
    a.L = c->L;
    a.col_begin = col_begin;
    a.col_step = col_step;
    a.col_end = col_end;
    a.nsweep = nsweep;
    a.W = W;
    a.vs = c->sweep_vs;
    a.variant = 1;  // nontemporal stores
    const int fc = c->cfg.flux_column - c->x_begin;
    a.flux_col = (fc >= 0 && fc < c->ncol) ? fc : -1;
    a.fskip0 = a.fskip1 = 0;
    a.flux_norm = c->cfg.flux_norm;
    a.Q = c->d_Q;
    a.c = c->coef;
    a.k = c->kc;
    return a;
}
template Sweep2Args<double> sweep_args<double>(iblb_ctx*, int, int, int, int, int);
template Sweep2Args<float> sweep_args<float>(iblb_ctx*, int, int, int, int, int);

// No IB force owed before or between the iterations (no IB points, no cilia)
static bool sweep_ready(const iblb_ctx* c) {
    if (!c->sweep_on || c->phase != PH_RUN || c->cilia_on || ib_active(c) || c->ib_state != IB_NONE) return false;
    if (single_slab(c)) return c->ncol >= 2;
    return rccl_multi(c) && c->ncol >= 4;
}

template <typename T>
static int sweep_launch(iblb_ctx* c, const Sweep2Args<T>& a, bool ghost, hipStream_t st, bool timed, long long cells) {
    size_t ev = 0;
    int rc = timed ? ev_begin(c, &ev, st) : IBLB_OK;
    if (rc) return rc;
    HIP_TRY(c, launch_sweep2<T>(a, ghost, st));
    return timed ? ev_end(c, ev, EV_SWEEP, cells, st) : IBLB_OK;
}

static void after_sweep(iblb_ctx* c, int K) {
    c->cur = 1 - c->cur;
    c->t += K;
    c->ghost = 0;
}

// Two iterations per launch.  A lone slab: one launch.  A slab of an RCCL group (>= 4 columns):
//   comm:    exchange(t, 2 columns) -> wait int(t-2) -> boundary sweeps [0, 2), [ncol-2, ncol)(t) -> ev_bnd
//   compute: (join_comm: boundary(t-2)) -> interior [2, ncol-2)(t) -> ev_int
// (IBLB_OVERLAP=0: everything on the compute stream, in sequence.)
template <typename T>
static int sweep_step(iblb_ctx* c) {
    const int W = std::max(1, c->sweep_w);
    if (single_slab(c)) {
        int rc = sweep_launch<T>(c, sweep_args<T>(c, 0, W, c->ncol, (c->ncol + W - 1) / W, W), false, c->stream, true,
                                 (long long)c->ncol * c->ny);
        if (rc) return rc;
        after_sweep(c, 2);
        return IBLB_OK;
    }
    int rc = join_comm(c);
    if (rc) return rc;
    const bool ov = c->overlap;
    hipStream_t bs = ov ? c->comm_stream : c->stream;
    if (ov && (rc = comm_ready(c, 2))) return rc;
    if ((rc = exchange(c, bs, 2))) return rc;
    if (ov && (rc = int_event(c))) return rc;
    if (ov) HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_int, 0));
    if ((rc = sweep_launch<T>(c, sweep_args<T>(c, 0, c->ncol - 2, c->ncol, 2, 2), true, bs, false, 0))) return rc;
    if (ov) HIP_TRY(c, hipEventRecord(c->ev_bnd, bs));
    const int ni = c->ncol - 4;
    if (ni > 0 && (rc = sweep_launch<T>(c, sweep_args<T>(c, 2, W, c->ncol - 2, (ni + W - 1) / W, W), false, c->stream,
                                        true, (long long)ni * c->ny)))
        return rc;
    if (ov) {
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        c->bnd_w = 2;
    } else if ((rc = comm_follows(c))) {
        return rc;
    }
    after_sweep(c, 2);
    return IBLB_OK;
}

// K = d iterations in one launch on a lone slab
template <typename T>
static int sweepk_step(iblb_ctx* c, int d) {
    const int W = std::max(1, c->deep_w);
    // balanced sweep widths (col_step 0: the launcher sizes the sweeps to whole rounds of waves)
    Sweep2Args<T> a = sweep_args<T>(c, 0, c->deep_balance ? 0 : W, c->ncol, (c->ncol + W - 1) / W, W);
    a.vs = c->deep_vs;
    a.variant = c->deep_variant;
    size_t ev = 0;
    hipEvent_t e0, e1;  // timing on the launch's own signals (profiling only)
    int rc = ev_kernel(c, &ev, &e0, &e1);
    if (rc) return rc;
    a.kinfo = c->deep_kinfo;
    HIP_TRY(c, launch_sweepk<T>(a, d, false, c->stream, e1, e0));
    if ((rc = ev_kernel_end(c, ev, EV_SWEEPK, (long long)c->ncol * c->ny))) return rc;
    after_sweep(c, d);
    c->deep_launches++;
    c->deep_iterations += d;
    return IBLB_OK;
}

// K = d iterations per cycle on a slab of an RCCL group (ncol >= 2K): K ghost columns
// exchanged and the boundary sweeps (output columns [0, K) and [ncol-K, ncol), which read columns
// -K .. 2K-1 and ncol-2K .. ncol+K-1) on the comm stream beside the interior sweep [K, ncol-K):
//   compute: (join_comm: boundary(t-K)) -> interior(t) -> ev_int
//   comm:    exchange(t) -> wait interior(t-K) (it read the columns boundary(t) overwrites) ->
//            boundary(t) -> ev_bnd
// The host submits the interior first: the launch the cycle time depends on leaves the host before
// the RCCL group and the boundary launch.  The interior and boundary launches signal ev_int / ev_bnd
// with their own completion signals (no marker packets: each cross-queue packet idles a queue for
// microseconds, profiles/r02q_*); the interior's event alternates between ev_int and ev_int2, so
// the comm stream's waits still name interior(t-K) while interior(t) is in flight.
// (IBLB_OVERLAP=0: exchange, boundary and interior in sequence on the compute stream.)
// K may differ from the previous cycle's (deep_depth): the exchange waits for the previous interior
// when it sends columns that interior wrote (comm_ready: K > bnd_w), and every ghost column read is
// within gc = 3 sweep_depth.
// Device handshake (round 5, IBLB_EDGE_FLAG=1 default).  Only the interior's first and last sweeps
// (its edge waves) touch what the comm stream's boundary sweeps touch: they pull columns [0, K) /
// [ncol-K, ncol) that boundary(t-K) wrote and overwrite [K, 2K) / [ncol-2K, ncol-K) that it read;
// boundary(t+K) in turn reads what they write and overwrites what they read.  So in a chain of
// cycles neither stream waits for the other in its queue:
//   - interior(t)'s edge waves poll a word that a signal kernel after boundary(t-K) sets
//     (launch_seq_signal) — the compute queue's barrier packet for ev_bnd cost ~9 us per cycle
//     (profiles/r04/bsplit, r05/edge);
//   - interior(t) carries no completion event (any signal on it, kernel's own or a marker, cost ~5 us
//     before the next interior, profiles/r05/gap); its edge waves count themselves into a second word
//     when their stores are released (lbm_sweep_impl.h:edge_done), and boundary(t+K)'s waves poll it
//     for the count interior(t) brings it to.
// Both polls are bounded (lbm_sweep_impl.h:edge_wait).  Every other interior wave starts and ends
// freely.  The interior is launched as a ghost-column build (it reads no ghost column: the same cells,
// addressed without the periodic wrap).  Edge waves: outputs below lo = 2 sweep_depth + 2 or above
// ncol - lo (every depth K - 1, K a call mixes).  Consumers of ev_int after the chain record it first
// (int_unrec: the compute stream's last work is then that interior).  Deadlock freedom with shared
// hardware queues: DESIGN.md §8 (the wait graph).
// (no reserved CUs: the spinning waves could hold the slots the other stream's kernels need — off)
static bool dev_handshake(const iblb_ctx* c) {
    return c->overlap && c->edge_flag && c->sig && c->reserved_cus > 0;
}
// IBLB_EDGE_FLAG=2: one way only (the interior's edge waves wait on the device word; the comm stream
// waits for the interior's completion event in its queue) — round 5's first step, kept for A/B
static bool one_way(const iblb_ctx* c) { return c->edge_flag == 2; }

// ev_int names the compute stream's last interior; after a handshake chain it is recorded on demand
static int int_event(iblb_ctx* c) {
    if (c->int_unrec) {
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        c->int_unrec = false;
    }
    return IBLB_OK;
}

template <typename T>
static int deep_slab_step(iblb_ctx* c, int K) {
    const int W = std::max(1, c->deep_w);
    const bool ov = c->overlap;
    const bool chained = ov && c->deep_chain && c->deep_chain_t == c->t && c->deep_chain_cur == c->cur;
    const bool hs = dev_handshake(c);
    const bool flag = chained && hs;  // device waits in both directions (else queue waits)
    const int lo = 2 * c->sweep_depth + 2, hi = c->ncol - lo;
    int rc = flag ? IBLB_OK : join_comm(c);
    if (rc) return rc;
    hipStream_t bs = ov ? c->comm_stream : c->stream;
    const int ni = c->ncol - 2 * K;  // interior [K, ncol-K): needs nothing from the halo
    const unsigned done_prev = c->done_n;  // the edge count interior(t-K) brought the done word to
    auto interior = [&](hipEvent_t stop) -> int {
        if (ni <= 0) {
            if (stop) HIP_TRY(c, hipEventRecord(stop, c->stream));
            return IBLB_OK;
        }
        Sweep2Args<T> a = sweep_args<T>(c, K, c->deep_balance ? 0 : W, c->ncol - K, (ni + W - 1) / W, W);
        a.vs = c->slab_vs;
        a.cus = c->ncu - c->reserved_cus;  // the compute stream's CU mask
        a.variant = c->int_variant >= 0 ? c->int_variant : c->deep_variant;
        int nedge = 0;
        if (hs) {
            a.wait_lo = lo;
            a.wait_hi = hi;
            a.edge_trim = c->edge_trim;
            if (!one_way(c)) {
                a.done_cnt = c->sig + 16;  // (the done word: its own 64-byte line)
                a.edge_waves = &nedge;
            }
            if (flag) {  // the value boundary(t-K)'s signal kernel stores
                a.wait_seq = c->sig;
                a.wait_val = c->sig_n;
                a.wait_err = c->sig_err;
                a.wait_ticks = c->wait_ticks;
                c->dev_wait_launches++;
            }
        }
        size_t ev = 0;
        hipEvent_t e0, e1;  // timing on the launch's own signals (profiling only)
        int r = ev_kernel(c, &ev, &e0, &e1);
        if (r) return r;
        a.kinfo = c->deep_kinfo;
        HIP_TRY(c, launch_sweepk<T>(a, K, hs, c->stream, e1 ? e1 : stop, e0));
        if (e1 && stop) HIP_TRY(c, hipEventRecord(stop, c->stream));
        c->done_n += (unsigned)nedge;
        return ev_kernel_end(c, ev, EV_SWEEPK, (long long)ni * c->ny);
    };
    auto boundary = [&](hipEvent_t stop) -> int {
        Sweep2Args<T> b = sweep_args<T>(c, 0, c->ncol - K, c->ncol, 2, K);  // [0, K) and [ncol-K, ncol)
        b.vs = c->slab_vs;
        b.variant = c->deep_variant;
        if (flag && !one_way(c)) {  // every wave waits for interior(t-K)'s edge waves
            b.wait_seq = c->sig + 16;
            b.wait_val = done_prev;
            b.wait_lo = INT_MAX;
            b.wait_hi = INT_MAX;
            b.wait_err = c->sig_err;
            b.wait_ticks = c->wait_ticks;
            c->dev_wait_launches++;
        }
        HIP_TRY(c, launch_sweepk<T>(b, K, true, bs, stop));
        return IBLB_OK;
    };
    if (!ov) {
        if ((rc = exchange(c, bs, K)) || (rc = boundary(nullptr)) || (rc = interior(nullptr))) return rc;
        if ((rc = comm_follows(c))) return rc;
        c->deep_chain = false;
    } else {
        // prev: the compute stream's work before interior(t) (interior(t-K) when chained)
        hipEvent_t prev = c->ev_int, next = c->ev_int2;
        if (!chained) {
            HIP_TRY(c, hipEventRecord(prev, c->stream));
            c->int_unrec = false;
        } else if (c->int_unrec && K > c->bnd_w) {  // the exchange below sends columns interior(t-K) wrote
            if ((rc = int_event(c))) return rc;
        }
        const bool two = hs && !one_way(c);
        if ((rc = interior(two ? nullptr : next))) return rc;
        if ((rc = comm_ready(c, K))) return rc;  // (waits for c->ev_int = prev)
        if ((rc = exchange(c, bs, K))) return rc;
        if (!(flag && two)) HIP_TRY(c, hipStreamWaitEvent(bs, prev, 0));
        if ((rc = boundary(c->ev_bnd))) return rc;
        if (hs) HIP_TRY(c, launch_seq_signal(c->sig, ++c->sig_n, bs));
        if (two) {
            c->int_unrec = true;  // ev_int (= prev) is recorded when someone needs it
        } else {
            c->ev_int = next;
            c->ev_int2 = prev;
        }
        c->bnd_w = K;
        c->deep_chain = true;
    }
    after_sweep(c, K);
    c->deep_launches++;
    c->deep_iterations += K;
    c->deep_chain_t = c->t;
    c->deep_chain_cur = c->cur;
    return IBLB_OK;
}

// A device wait (deep_slab_step, band_step) that timed out leaves wrong populations behind: the call
// that ran it fails (the flag is read after the compute stream is synchronised).  With profiling on,
// the two-way handshake's done word is also checked against the edge-wave count the launcher
// computed on the host (launch_sweepk_mode's edge_waves): every interior has ended here.
int check_wait_err(iblb_ctx* c) {
    if (!c->sig_err) return IBLB_OK;
    if (__atomic_load_n(c->sig_err, __ATOMIC_ACQUIRE) != 0) {
        __atomic_store_n(c->sig_err, 0u, __ATOMIC_RELEASE);
        c->deep_chain = false;
        char msg[320];
        std::snprintf(msg, sizeof msg,
                      "a device-side wait of the slab hand-off exceeded the wait timeout (%g s, IBLB_WAIT_TIMEOUT_S / "
                      "iblb_set_wait_timeout): a neighbour rank or the comm stream stalled longer than that; the "
                      "state is invalid (set it again)",
                      c->wait_timeout_s);
        return fail(c, IBLB_ERR_COMM, msg);
    }
    if (c->prof == 1 && c->sig && c->done_n) {  // (not in mode 2: the bench's timed regions)
        unsigned w = 0;
        HIP_TRY(c, hipMemcpy(&w, c->sig + 16, sizeof w, hipMemcpyDeviceToHost));
        if (w != c->done_n) {
            c->deep_chain = false;
            return fail(c, IBLB_ERR_COMM,
                        "slab hand-off: the done word (" + std::to_string(w) + ") differs from the edge waves launched (" +
                            std::to_string(c->done_n) + ")");
        }
    }
    return IBLB_OK;
}

int set_wait_ticks(iblb_ctx* c) {
    if (c->clock_hz <= 0.) {
        int khz = 0;
        HIP_TRY(c, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
        if (khz <= 0) return fail(c, IBLB_ERR_HIP, "the device reports no wall-clock rate");
        c->clock_hz = 1e3 * khz;
    }
    const double t = c->wait_timeout_s * c->clock_hz;
    c->wait_ticks = t >= 1.8e19 ? ~0ull : (unsigned long long)t;
    return IBLB_OK;
}

int hold_release(iblb_ctx* c) {
    if (c->hold_thread.joinable()) c->hold_thread.join();
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

static int step_one(iblb_ctx* c) {
    int rc = join_comm(c);
    if (rc) return rc;
    if (c->cilia_on && !c->cil_sched) {
        if (c->phase == PH_RUN && ((rc = ensure_halo(c)) || (rc = ensure_force(c)))) return rc;
        if ((rc = run_cilia(c))) return rc;
    } else if (c->phase == PH_RUN && rccl_multi(c) && c->overlap && c->ib_state == IB_PENDING && c->ghost < 3 &&
               c->ncol >= 9) {
        const int next = c->sch_n > 0 && sched_entry(c, c->t) != c->sch_cur ? sched_entry(c, c->t) : -1;
        return is_f64(c) ? ib_overlapped_step<double>(c, next) : ib_overlapped_step<float>(c, next);
    } else if (c->sch_n > 0 && sched_entry(c, c->t) != c->sch_cur) {
        // the force owed to the previous iteration's points first, then this iteration's points
        if (c->phase == PH_RUN && ((rc = ensure_halo(c)) || (rc = ensure_force(c)))) return rc;
        sched_use(c, sched_entry(c, c->t));
    }
    if (c->phase == PH_RUN && rccl_multi(c) && c->overlap && c->ghost == 0 && c->ib_state != IB_PENDING &&
        c->ncol >= 3)
        return is_f64(c) ? overlapped_step<double>(c) : overlapped_step<float>(c);
    if (c->phase == PH_RUN && ((rc = ensure_halo(c)) || (rc = ensure_force(c)))) return rc;
    if ((rc = advance(c))) return rc;
    if (c->phase == PH_RUN && c->t == 1 && c->rho0) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        free_boot(c);
    }
    return IBLB_OK;
}

// Make ghosts and force^t of the current state available to a reader.
int prepare_read(iblb_ctx* c) {
    int rc = check_ready(c);
    if (rc) return rc;
    if (c->phase != PH_RUN) return IBLB_OK;
    if ((rc = join_comm(c))) return rc;
    if (c->transport == TR_LOCAL) {
        if (c->ghost < 1 || c->ib_state == IB_PENDING)
            return fail(c, IBLB_ERR_STATE, "local group state not prepared (use iblb_group_step)");
        return IBLB_OK;
    }
    if ((rc = ensure_halo(c))) return rc;
    return ensure_force(c);
}

}  // namespace iblbh

using namespace iblbh;

extern "C" {

// Depth of the next deep launch without IB, r >= K-1 iterations left in the call: K, or K-1 where
// launches of K-1 (j of them) leave a multiple of K, so that r = j (K-1) + m K needs no two-iteration
// or one-step remainder (every r >= (K-1)(K-2) qualifies: 20 = 4 x 5 at K = 6, 500 = 4 x 5 + 80 x 6).
// A remainder costs more than the depth: M f64 20 iterations at K = 6 as 3 x 6 + 2 took 0.111 ms per
// iteration against 0.097 as 4 x 5 (profiles/r04/depth).
static int deep_depth(const iblb_ctx* c, int r) {
    const int K = c->sweep_depth;
    if (K < 4) return K;
    const int j = (K - r % K) % K;
    return (j > 0 && (long)j * (K - 1) <= r) ? K - 1 : K;
}

// nsteps iterations by the fastest applicable schedule per iteration (band cycles, deep sweeps,
// two-iteration sweeps, one-step iterations); the band streams may still run at the end
static int step_range(iblb_ctx* c, int nsteps) {
    int rc = IBLB_OK;
    const int K = c->sweep_depth;
    for (int s = 0; s < nsteps;) {
        if (nsteps - s >= K && c->phase == PH_RUN && (!c->cilia_on || c->cil_sched) && K >= 3) {
            // a schedule's cycle whose plan was declined (trapezoids over half the lattice) is
            // planned again K iterations later, not at every one-step iteration in between
            if (c->sch_n > 0 && c->t >= c->band_retry_t) {
                if (!(rc = plan_cycle(c)) && !c->band_valid) c->band_retry_t = c->t + K;
            } else if (c->band_dirty) {
                rc = plan_bands(c, c->pts_host);
            }
            if (rc) return rc;
        }
        if (nsteps - s >= K && band_ready(c)) {
            if ((rc = band_step_any(c))) return rc;
            s += K;
            continue;
        }
        if ((rc = band_join(c))) return rc;
        const int d = nsteps - s >= K - 1 ? deep_depth(c, nsteps - s) : K;
        if (d >= 3 && nsteps - s >= d && sweep_ready(c)) {
            if (single_slab(c)) {
                if ((rc = is_f64(c) ? sweepk_step<double>(c, d) : sweepk_step<float>(c, d))) return rc;
                s += d;
                continue;
            }
            if (rccl_multi(c) && c->ncol >= 2 * d) {
                if ((rc = is_f64(c) ? deep_slab_step<double>(c, d) : deep_slab_step<float>(c, d))) return rc;
                s += d;
                continue;
            }
        }
        if (nsteps - s >= 2 && sweep_ready(c)) {
            if ((rc = is_f64(c) ? sweep_step<double>(c) : sweep_step<float>(c))) return rc;
            s += 2;
            continue;
        }
        if ((rc = step_one(c))) return rc;
        ++s;
    }
    return IBLB_OK;
}

int iblb_step(iblb_ctx* c, int nsteps) {
    if (!c || nsteps < 0) return IBLB_ERR_ARG;
    if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: use iblb_group_step");
    int rc = check_ready(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    const int K = c->sweep_depth;
    // on-device cilia: the kinematics of up to CILIA_AHEAD iterations run ahead as a schedule, so
    // that the band cycle applies (cilia_schedule); otherwise one kinematics launch per iteration
    constexpr int CILIA_AHEAD = 500;
    for (int done = 0; done < nsteps;) {
        int seg = nsteps - done;
        if (c->cilia_on && seg >= K && band_possible(c)) {
            seg = std::min(seg, CILIA_AHEAD);
            if ((rc = cilia_schedule(c, seg)) || (rc = step_range(c, seg)) || (rc = cilia_schedule_end(c))) return rc;
        } else if ((rc = step_range(c, seg))) {
            return rc;
        }
        done += seg;
    }
    if ((rc = band_join(c))) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return check_wait_err(c);
}

// ---- local groups -------------------------------------------------------------------------------
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
        ctxs[i]->ghost = 0;
        ctxs[i]->band_valid = false;
    }
    return sync_all(ctxs, n);
}

// ghost columns of every slab from its neighbours' current buffers (three with an owed IB force)
static int group_exchange(iblb_ctx** cs, int n) {
    bool ib = false;
    for (int i = 0; i < n; ++i) ib |= cs[i]->ib_state == IB_PENDING;
    const int d = ib ? 3 : 1;
    int rc = sync_all(cs, n);
    if (rc) return rc;
    for (int i = 0; i < n; ++i) {
        iblb_ctx* c = cs[i];
        if (d > c->left->ncol || d > c->right->ncol) return fail(c, IBLB_ERR_ARG, "slab narrower than its halo");
        HIP_TRY(c, hipSetDevice(c->device));
        const size_t cb = (size_t)c->L.col * c->esize;
        char* g = (char*)c->g[c->cur];
        const char* gl = (const char*)c->left->g[c->left->cur];
        const char* gr = (const char*)c->right->g[c->right->cur];
        HIP_TRY(c, hipMemcpyAsync(g - (size_t)d * cb, gl + (size_t)(c->left->ncol - d) * cb, (size_t)d * cb,
                                  hipMemcpyDefault, c->stream));
        HIP_TRY(c, hipMemcpyAsync(g + (size_t)c->ncol * cb, gr, (size_t)d * cb, hipMemcpyDefault, c->stream));
    }
    if ((rc = sync_all(cs, n))) return rc;
    for (int i = 0; i < n; ++i) cs[i]->ghost = d;
    return IBLB_OK;
}

static int group_force(iblb_ctx** cs, int n) {
    int rc;
    for (int i = 0; i < n; ++i) {
        iblb_ctx* c = cs[i];
        if (c->ib_state != IB_PENDING) continue;
        if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
        HIP_TRY(c, hipSetDevice(c->device));
        if ((rc = ib_ghost(c, c->g[c->cur], c->ghost, 0, c->ncol, pts_s(c), pts_us(c), pts_eps(c), 0, c->stream)))
            return rc;
        c->ib_state = IB_READY;
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
            const int need = cs[0]->ib_state == IB_PENDING ? 3 : 1;
            if (cs[0]->ghost < need && (rc = group_exchange(cs, n))) return rc;
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
    // leave the group readable: ghosts of the new state and its force^t
    if ((rc = group_exchange(cs, n))) return rc;
    if ((rc = group_force(cs, n))) return rc;
    for (int i = 0; i < n; ++i)
        if (cs[i]->phase == PH_RUN && cs[i]->t >= 1 && cs[i]->rho0) free_boot(cs[i]);
    return sync_all(cs, n);
}

// ---- RCCL groups --------------------------------------------------------------------------------
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
    c->deep_chain = false;
    if (c->transport != TR_NONE) return fail(c, IBLB_ERR_STATE, "context already linked");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    NCCL_TRY(c, ncclCommInitRank(&c->comm, nranks, u, rank));
    c->nranks = nranks;
    c->rank = rank;
    c->transport = TR_RCCL;
    // IBLB_RCCL_SELF=1 with one rank: the slab exchanges its ghosts with itself through RCCL, so the
    // multi-slab schedule (comm stream, overlap, all-reduces) runs on one GPU
    c->self_ring = nranks == 1 && env_long("IBLB_RCCL_SELF", 0) != 0;
    if (nranks > 1) {
        // the slabs must tile the lattice in rank order: check (x_begin, ncol) of all ranks
        void* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, 2 * sizeof(int) * (size_t)nranks));
        int mine[2] = {c->x_begin, c->ncol};
        hipError_t e = hipMemcpy((int*)d + 2 * rank, mine, sizeof(mine), hipMemcpyHostToDevice);
        ncclResult_t r = e == hipSuccess ? ncclAllGather((int*)d + 2 * rank, d, 2, ncclInt32, c->comm, c->stream)
                                         : ncclSuccess;
        std::vector<int> all(2 * (size_t)nranks);
        if (e == hipSuccess && r == ncclSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess && r == ncclSuccess) e = hipMemcpy(all.data(), d, all.size() * sizeof(int), hipMemcpyDeviceToHost);
        (void)hipFree(d);
        HIP_TRY(c, e);
        NCCL_TRY(c, r);
        long total = 0;
        for (int q = 0; q < nranks; ++q) {
            total += all[2 * q + 1];
            const int nxt = (q + 1) % nranks;
            if ((all[2 * q] + all[2 * q + 1]) % c->nx != all[2 * nxt])
                return fail(c, IBLB_ERR_ARG, "RCCL group: slabs must tile the lattice in rank order");
        }
        if (total != c->nx) return fail(c, IBLB_ERR_ARG, "RCCL group: slabs do not cover the lattice");
        c->slab_begin.resize(nranks);
        c->slab_count.resize(nranks);
        for (int q = 0; q < nranks; ++q) {
            c->slab_begin[q] = all[2 * q];
            c->slab_count[q] = all[2 * q + 1];
        }
    } else {
        if (c->self_ring && c->ncol != c->nx) return fail(c, IBLB_ERR_ARG, "IBLB_RCCL_SELF needs the whole lattice");
        c->slab_begin.assign(1, c->x_begin);
        c->slab_count.assign(1, c->ncol);
    }
    c->min_slab = *std::min_element(c->slab_count.begin(), c->slab_count.end());
    if (rccl_multi(c)) {
        // The compute stream gets a CU mask that leaves whole columns of CUs (the top mask bits: bit
        // i is a CU of XCD i % 8, so 8m bits are m CUs of every XCD, profiles/r02n_xcc_probe.txt) to
        // the comm stream: enough for every wave of the two boundary sweeps to be resident at once,
        // rounded up to a multiple of the XCD count (32 measured best at 4096 rows: self ring
        // 512 / 1024 / 2048 x 4096 0.0376 / 0.0564 / 0.0953 ms/iteration vs 0.046 / 0.080 / 0.148
        // with 16, profiles/r01e5_gap_probe_reserve.txt).  IBLB_RESERVE_CUS overrides (0 = none).
        hipDeviceProp_t prop;
        HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
        c->ncu = prop.multiProcessorCount;
        long reserve = 8;
        if (c->sweep_depth >= 3) {
            int nch = 0;
            const int wpc = is_f64(c) ? sweepk_geometry<double>(c->sweep_depth, c->slab_vs, c->deep_variant, true, c->ny, &nch)
                                      : sweepk_geometry<float>(c->sweep_depth, c->slab_vs, c->deep_variant, true, c->ny, &nch);
            if (wpc > 0) {
                const long need = std::max(8L, (long)((2 * nch + wpc - 1) / wpc));
                const long xcd = std::max(1, c->ncu / 8);
                reserve = std::min((long)c->ncu / 2, (need + xcd - 1) / xcd * xcd);
            }
        }
        reserve = env_long("IBLB_RESERVE_CUS", reserve);
        if (reserve >= c->ncu) return fail(c, IBLB_ERR_ARG, "IBLB_RESERVE_CUS exceeds the compute units");
        if (reserve > 0) {
            const int ncu = c->ncu;
            std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u), rest(mask.size(), 0u);
            for (int i = 0; i < ncu; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
            for (long k = 0; k < reserve; ++k) {
                const long i = ncu - 1 - k;
                mask[(size_t)i / 32] &= ~(1u << (i % 32));
                rest[(size_t)i / 32] |= 1u << (i % 32);
            }
            hipStream_t masked = nullptr;
            HIP_TRY(c, hipExtStreamCreateWithCUMask(&masked, (uint32_t)mask.size(), mask.data()));
            c->reserved_cus = (int)reserve;
            c->comp_mask = mask;
            (void)hipStreamDestroy(c->stream);
            c->stream = masked;
            // the comm stream confined to the reserved CUs: a boundary sweep dispatched before the
            // interior of the same cycle must not take CUs the interior's round of waves needs
            HIP_TRY(c, hipExtStreamCreateWithCUMask(&c->comm_stream, (uint32_t)rest.size(), rest.data()));
        } else {
            int prio_lo = 0, prio_hi = 0;
            HIP_TRY(c, hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
            HIP_TRY(c, hipStreamCreateWithPriority(&c->comm_stream, hipStreamNonBlocking, prio_hi));
        }
        // cross-stream ordering events (producer and consumer on this device): no system-scope
        // fence (512 x 4096 self ring 0.0394 vs 0.0420 ms/iteration, profiles/r01u_gap_probe_event_fence.txt)
        const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
        for (hipEvent_t* e : {&c->ev_bnd, &c->ev_int, &c->ev_int2, &c->ev_pre, &c->ev_x, &c->ev_rccl})
            HIP_TRY(c, hipEventCreateWithFlags(e, evf));
        HIP_TRY(c, hipEventRecord(c->ev_bnd, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));
        c->overlap = env_long("IBLB_OVERLAP", 1) != 0;
        // one way in f64 (512 x 4096 self ring 0.01502-0.01506 vs 0.01517-0.0152 two-way: the edge waves'
        // write-through stores cost what the interior's event did), two-way in f32 (1024 x 2048: 0.01094-
        // 0.0110 vs 0.01125), profiles/r05/hs3
        c->edge_flag = (int)env_long("IBLB_EDGE_FLAG", is_f64(c) ? 2 : 1);
        c->int_variant = (int)env_long("IBLB_INTERIOR_VARIANT", -1);
        c->edge_trim = (int)std::max(0L, env_long("IBLB_EDGE_TRIM", 0));
        if (!c->sig) {
            int rc = alloc_zero(c, (void**)&c->sig, 128);  // signal word, done word (+64 B)
            if (rc) return rc;
            HIP_TRY(c, hipHostMalloc((void**)&c->sig_err, 64, hipHostMallocCoherent));
            *c->sig_err = 0;
            c->sig_n = 0;
            c->done_n = 0;
        }
        if (int rc = set_wait_ticks(c)) return rc;
        // IBLB_TEST_HOLD=<n>:<ms> (tests): exchange n since this attach starts ms milliseconds late
        if (const char* h = std::getenv("IBLB_TEST_HOLD")) {
            long long n = -1;
            int ms = 0;
            if (std::sscanf(h, "%lld:%d", &n, &ms) != 2 || n < 0 || ms < 0)
                return fail(c, IBLB_ERR_ARG, "IBLB_TEST_HOLD: expected <exchange>:<milliseconds>");
            if (!c->hold_word) {
                HIP_TRY(c, hipHostMalloc((void**)&c->hold_word, 64, hipHostMallocCoherent));
                *c->hold_word = 0;
            }
            c->hold_x = n;
            c->hold_ms = ms;
        }
        c->n_exch = 0;
        c->bnd_w = INT_MAX;
        c->rccl_last = nullptr;  // the attach's all-gather is complete (synchronised above)
    }
    c->ghost = 0;
    c->band_valid = false;
    c->band_dirty = c->sch_n == 0 && ib_active(c) && !c->cilia_on;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return IBLB_OK;
}

}  // extern "C"
