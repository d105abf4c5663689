// iblb_ctx.hip — the fused context API of include/iblb.h: lifecycle, state, Lagrangian points,
// readers in the reference layouts, the output gather and checkpoint / restart.  Time stepping is
// in ctx_step.hip, the IB band cycle in ctx_band.hip; the context itself in ctx.h.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ctx.h"

namespace iblbh {

std::string g_create_error;

long env_long(const char* name, long dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::strtol(v, nullptr, 10) : dflt;
}

int fail(iblb_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    else g_create_error = msg;
    return code;
}

int hip_fail(iblb_ctx* c, hipError_t e, const char* what) {
    return fail(c, e == hipErrorOutOfMemory ? IBLB_ERR_NOMEM : IBLB_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// ---- profiling ----------------------------------------------------------------------------------
static void ev_account(iblb_ctx* c, const iblb_ctx::EvRec& r, float ms) {
    if (r.kind == EV_FUSED) { c->fused_ms += ms; c->fused_launches++; c->fused_cells += r.cells; }
    else if (r.kind == EV_SWEEP) { c->sweep_ms += ms; c->sweep_launches++; c->sweep_cells += r.cells; }
    else if (r.kind == EV_SWEEPK) { c->sweepk_ms += ms; c->sweepk_launches++; c->sweepk_cells += r.cells; }
    else if (r.kind == EV_IB) c->ib_ms += ms;
    else c->halo_ms += ms;
}

static int ev_drain(iblb_ctx* c) {
    for (auto& r : c->ev_kind) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev_pool[r.idx], c->ev_pool[r.idx + 1]));
        ev_account(c, r, ms);
    }
    c->ev_kind.clear();
    c->ev_used = 0;
    return IBLB_OK;
}

static int ev_reserve(iblb_ctx* c, size_t* idx) {
    if (c->ev_used + 2 > c->ev_pool.size()) {
        // timing events bracket kernels of this device only: no system-scope fence
        for (int k = 0; k < 64; ++k) {
            hipEvent_t e;
            HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
            c->ev_pool.push_back(e);
        }
    }
    *idx = c->ev_used;
    c->ev_used += 2;
    return IBLB_OK;
}

int ev_begin(iblb_ctx* c, size_t* idx, hipStream_t st) {
    if (c->prof != 1) return IBLB_OK;  // (mode 2: only the deep launches' own signals)
    int rc = ev_reserve(c, idx);
    if (rc) return rc;
    HIP_TRY(c, hipEventRecord(c->ev_pool[*idx], st ? st : c->stream));
    return IBLB_OK;
}

static int ev_note(iblb_ctx* c, size_t idx, int kind, long long cells) {
    c->ev_kind.push_back({kind, idx, cells});
    if (c->ev_used >= 8192) {  // bound the pool: drain what is recorded
        HIP_TRY(c, hipEventSynchronize(c->ev_pool[idx + 1]));
        for (hipStream_t s : {c->stream, c->comm_stream, c->band_st, c->deep_st})
            if (s) HIP_TRY(c, hipStreamSynchronize(s));
        return ev_drain(c);
    }
    return IBLB_OK;
}

int ev_end(iblb_ctx* c, size_t idx, int kind, long long cells, hipStream_t st) {
    if (c->prof != 1) return IBLB_OK;
    HIP_TRY(c, hipEventRecord(c->ev_pool[idx + 1], st ? st : c->stream));
    return ev_note(c, idx, kind, cells);
}

int ev_kernel(iblb_ctx* c, size_t* idx, hipEvent_t* start, hipEvent_t* stop) {
    *start = *stop = nullptr;
    if (!c->prof) return IBLB_OK;
    int rc = ev_reserve(c, idx);
    if (rc) return rc;
    *start = c->ev_pool[*idx];
    *stop = c->ev_pool[*idx + 1];
    return IBLB_OK;
}

int ev_kernel_end(iblb_ctx* c, size_t idx, int kind, long long cells) {
    if (!c->prof) return IBLB_OK;
    return ev_note(c, idx, kind, cells);
}

// ---- allocation ---------------------------------------------------------------------------------
// Allocation zeroed on the context's (non-blocking) stream, so later work on that stream is
// ordered after the clear.
int alloc_zero(iblb_ctx* c, void** p, size_t bytes) {
    HIP_TRY(c, hipMalloc(p, bytes));
    HIP_TRY(c, hipMemsetAsync(*p, 0, bytes, c->stream));
    return IBLB_OK;
}

int free_boot(iblb_ctx* c) {
    for (double* p : {c->rho0, c->u0, c->force0})
        if (p) (void)hipFree(p);
    c->rho0 = c->u0 = c->force0 = nullptr;
    return IBLB_OK;
}

// Scratch device buffer freed at scope exit.
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

static size_t round_up(size_t v, size_t m) { return (v + m - 1) / m * m; }

// rho [N] and u [2N] of the slab in the reference layout (j = y*ncol + xc), into device buffers,
// on the context's stream.  The state must be prepared (prepare_read).
static int macro_device(iblb_ctx* c, double* dr, double* du) {
    if (c->phase == PH_BOOT) {
        HIP_TRY(c, launch_field_out(c->rho0, dr, c->L, 1, c->fplane, 0., 0., c->stream));
        HIP_TRY(c, launch_field_out(c->u0, du, c->L, 2, c->fplane, 0., 0., c->stream));
        return IBLB_OK;
    }
    const double* fd = c->ib_state == IB_READY ? c->fdense : nullptr;
    if (is_f64(c))
        HIP_TRY(c, launch_macro_out<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), fd, c->fplane,
                                            c->coef.gx, c->coef.gy, dr, du, c->stream));
    else
        HIP_TRY(c, launch_macro_out<float>(gptr<float>(c, c->cur), c->L, halo_of<float>(c, c->cur), fd, c->fplane,
                                           c->coef.gx, c->coef.gy, dr, du, c->stream));
    return IBLB_OK;
}

static std::vector<float> host_points(const float* s, size_t ns) { return std::vector<float>(s, s + 2 * ns); }

// The points about to be replaced: any force still owed to them is evaluated first (collective in
// an RCCL group), after the comm stream's work of the last step (a one-step IB on the
// comm stream may still read the schedule arrays, and an RCCL exchange there must precede this
// one); afterwards the arrays may be rewritten on the context's stream.
int retire_points(iblb_ctx* c) {
    int rc = join_comm(c);
    if (rc) return rc;
    if (c->ib_state == IB_PENDING) {
        if (c->transport == TR_LOCAL) return fail(c, IBLB_ERR_STATE, "local group: set points between group steps");
        if ((rc = ensure_force(c))) return rc;
    }
    // the points of an active schedule entry become the static points (readers and checkpoints
    // between this call and the next step see them)
    if (c->sch_n > 0 && c->sch_cur >= 0 && c->ns > 0) {
        const size_t ns = (size_t)c->ns;
        HIP_TRY(c, hipMemcpyAsync(c->d_s, pts_s(c), 2 * ns * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->d_us, pts_us(c), 2 * ns * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->d_eps, pts_eps(c), ns * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
        const size_t e = (size_t)c->sch_cur;
        c->pts_host.assign(c->sch_x.begin() + e * 2 * ns, c->sch_x.begin() + (e + 1) * 2 * ns);
    }
    c->sch_n = 0;
    c->sch_cur = -1;
    return IBLB_OK;
}

// device arrays of a schedule of n entries of the context's max_points
static int sched_reserve(iblb_ctx* c, size_t n, int ns) {
    if (n <= c->sch_cap && ns == c->ns) return IBLB_OK;
    for (void* p : {(void*)c->d_sch_s, (void*)c->d_sch_us, (void*)c->d_sch_eps})
        if (p) (void)hipFree(p);
    c->d_sch_s = c->d_sch_us = nullptr;
    c->d_sch_eps = nullptr;
    c->sch_cap = 0;
    const size_t cap = n * c->max_points;
    HIP_TRY(c, hipMalloc(&c->d_sch_s, 2 * cap * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->d_sch_us, 2 * cap * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->d_sch_eps, cap * sizeof(int)));
    c->sch_cap = n;
    return IBLB_OK;
}

// The reference's cilia kinematics (main.cu:822-841) of iterations t .. t+n-1 run ahead on the
// device into a schedule (the kinematics depend on `it` and on their own previous positions only,
// not on the fluid), so that iblb_step can take the IB band cycle with on-device cilia: one
// device-to-host copy of the n entries' positions for the cycles' band plans instead of the
// schedule upload of iblb_set_lagrangian_steps.  The schedule is retired (its last entry becomes
// the current points) when the n iterations are done (cilia_schedule_end).
int cilia_schedule(iblb_ctx* c, int n) {
    int rc = retire_points(c);  // the force owed to the current points first
    if (rc) return rc;
    const iblb_cilia& k = c->cilia;
    const int ns = CILIA_POINTS * k.c_num;
    c->sch_x_prev.clear();
    if (c->ns > 0 && c->ib_state == IB_READY) {  // a force from the current points is owed to iteration t
        c->sch_x_prev.resize(2 * (size_t)c->ns);
        HIP_TRY(c, hipMemcpyAsync(c->sch_x_prev.data(), c->d_s, 2 * (size_t)c->ns * sizeof(float), hipMemcpyDeviceToHost,
                                  c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if ((rc = sched_reserve(c, (size_t)n, ns))) return rc;
    const size_t per = (size_t)ns;  // entries packed at the points' count (sched_ptr)
    for (int i = 0; i < n; ++i) {
        const int it = (int)(c->t + i);
        HIP_TRY(c, launch_define_filament(k.T, it, k.c_space, k.p_step, (double)k.c_num, c->cil_samples, c->cil_lasts,
                                          c->cil_bpoints, c->stream));
        HIP_TRY(c, launch_boundary_check(k.c_space, k.c_num, c->nx, it, c->cil_bpoints, c->d_sch_s + 2 * per * i,
                                         c->d_sch_us + 2 * per * i, c->d_sch_eps + per * i, c->stream));
    }
    // the entries' (x, y) for the band plans
    c->sch_x.resize(2 * per * (size_t)n);
    HIP_TRY(c, hipMemcpyAsync(c->sch_x.data(), c->d_sch_s, c->sch_x.size() * sizeof(float), hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->ns = ns;
    c->sch_t0 = c->t;
    c->sch_n = n;
    c->sch_cur = -1;  // d_s holds the points before the schedule
    c->cil_sched = true;
    c->band_sticky = true;
    c->band_valid = false;
    c->band_retry_t = 0;
    c->band_dirty = false;
    return IBLB_OK;
}

int cilia_schedule_end(iblb_ctx* c) {
    if (!c->cil_sched) return IBLB_OK;
    c->cil_sched = false;
    int rc = band_join(c);
    if (rc) return rc;
    return retire_points(c);  // the last entry becomes the current points (d_s, for readers and the next call)
}

static int check_slab_points(iblb_ctx* c, size_t np, const float* s) {
    if (np == 0 || c->ncol == c->nx) return IBLB_OK;
    if (c->ncol < 3) return fail(c, IBLB_ERR_ARG, "immersed boundary across slabs needs >= 3 columns per slab");
    for (size_t k = 0; k < np; ++k) {
        const double x0 = std::nearbyint((double)s[2 * k]);
        if (!(x0 >= 0. && x0 <= (double)c->nx))
            return fail(c, IBLB_ERR_ARG, "slab groups need 0 <= nearbyint(s_x) <= XDIM (main.cu:202-205)");
    }
    return IBLB_OK;
}

}  // namespace iblbh

using namespace iblbh;

// ============================================================================================
extern "C" {

static int reset_cilia_state(iblb_ctx* c) {
    const size_t nk = (size_t)CILIA_SAMPLES * c->cilia.c_num;
    HIP_TRY(c, hipMemsetAsync(c->cil_samples, 0, 5 * nk * sizeof(float), c->stream));
    HIP_TRY(c, hipMemsetAsync(c->cil_lasts, 0, 2 * nk * sizeof(float), c->stream));
    HIP_TRY(c, hipMemsetAsync(c->cil_bpoints, 0, 5 * (size_t)CILIA_POINTS * c->cilia.c_num * sizeof(float), c->stream));
    return IBLB_OK;
}

const char* iblb_version(void) { return "iblb-mi355x 0.6 (gfx950, abi 6)"; }
int iblb_abi_version(void) { return IBLB_ABI_VERSION; }

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
    const bool f64 = c->prec == IBLB_PREC_F64;
    c->esize = f64 ? 8 : 4;
    c->V = f64 ? vec_of<double>() : vec_of<float>();
    c->nch = chunks_per_column(c->ny, c->V);
    c->device = cfg->device;
    c->max_points = cfg->max_points;
    // kernel defaults measured on MI355X: one-step variant f64 = DPP row shift +
    // nontemporal stores (5), f32 = nontemporal loads and stores (3); two-step sweeps 16 B per lane
    // (f64 2 cells, f32 4) over 4 / 6 columns; deep sweeps K = 7 (round 4, profiles/r04/depth: M f64
    // 171k / 174k / 182k MLUPS at K = 5 / 6 / 7, f32 255k / 280k / 304k; K = 8 dropped), 2 cells per
    // lane, ~96 (f64) / ~64
    // (f32) columns balanced to whole rounds of resident waves, the linear wave order dealt to the
    // XCDs in contiguous ranges (map 2) with alternate sweeps walking towards each other
    c->variant = (int)env_long("IBLB_FUSED_VARIANT", f64 ? 5 : 3);
    c->sweep_on = env_long("IBLB_SWEEP", 1) != 0;
    c->sweep_w = (int)env_long("IBLB_SWEEP_W", f64 ? 4 : 6);
    c->sweep_vs = (int)env_long("IBLB_SWEEP_VS", f64 ? 2 : 4);
    c->sweep_depth = (int)std::min(7L, std::max(2L, env_long("IBLB_SWEEP_DEPTH", 7)));
    c->deep_w = (int)env_long("IBLB_DEEP_W", f64 ? 96 : 64);
    c->deep_vs = (int)env_long("IBLB_DEEP_VS", 2);
    // f32: the wall split (variant bit 1) with the packed collide (bit 3), profiles/r04/pack, and on
    // one-cell group slabs the split with the preshift (bits 5, 6: 107 = 11 | 32 | 64; self ring
    // 512 x 4096 0.01158 vs 0.01242 ms/iteration, 2048 x 2048 0.0187 vs 0.0210, profiles/r04/depth);
    // f64: the wall split with the level-1 preshift (bits 1, 5: M f64 0.480 vs 0.521 ms per launch,
    // profiles/r04/split64) and the LDS window (bit 7: 163 = 35 | 128; M f64 0.621 vs 0.633 ms per
    // depth-7 launch, 512-column self ring 0.0159 vs 0.0163 ms/iteration, profiles/r04/ldswin)
    // f32, round 5: bit 7 on the packed two-cell walk keeps two of the three moving populations in LDS
    // (165 VGPRs: three waves per SIMD; 235 = 107 | 128): M f32 0.361 vs 0.387 ms per launch, 320k vs
    // 300k MLUPS, K5 249k vs 237k (profiles/r05/f32lw); group slabs (one cell per lane) ignore it
    c->deep_variant = (int)env_long("IBLB_DEEP_VARIANT", f64 ? 163 : 235);
    c->deep_balance = (int)env_long("IBLB_DEEP_BALANCE", 1);
    c->band_on = (int)env_long("IBLB_IB_BAND", 1);
    c->band_merge = (int)env_long("IBLB_BAND_MERGE", 1);
#ifdef IBLB_TIMING_PROBES
    // timing probes that skip work (WRONG results): only in a build made for them
    c->probe_level = (int)env_long("IBLB_PROBE_LEVEL", 0);
#else
    if (env_long("IBLB_PROBE_LEVEL", 0) != 0)
        std::fprintf(stderr, "iblb: IBLB_PROBE_LEVEL ignored: the library was built without IBLB_TIMING_PROBES\n");
#endif
    // the device waits' bound (ctx_step.hip:set_wait_ticks; iblb_set_wait_timeout overrides)
    if (const char* w = std::getenv("IBLB_WAIT_TIMEOUT_S")) {
        const double s = std::strtod(w, nullptr);
        if (s > 0.) c->wait_timeout_s = s;
    }
    c->band_deep_variant = (int)env_long("IBLB_BAND_DEEP_VARIANT", -1);
    c->wrap_split = (int)env_long("IBLB_WRAP_SPLIT", 1);
    c->band_par_env = (int)env_long("IBLB_BAND_PAR", 1);
    c->band_vhalf_env = (int)env_long("IBLB_BAND_VHALF", 1);
    // cells per lane in a group slab's deep sweeps: f64 two (the wall split needs them: self ring
    // 512 / 1024 / 2048 x 4096 0.0170 / 0.0293 / 0.0531 ms/iteration vs 0.0194 / 0.0343 / 0.0638
    // with one, profiles/r04/split64); f32 one (1024 / 2048 x 2048: 0.0126 / 0.0203 vs 0.0133 /
    // 0.0220 with two; round 1: profiles/r01e7_*)
    c->slab_vs = env_long("IBLB_SLAB_VS", f64 ? 2 : 1) == 2 ? 2 : 1;
    // ghost columns: K for a deep cycle's halo, 3 for a one-step IB halo, 3K for the IB band
    // trapezoids that cross a slab edge (ctx_band.hip)
    c->gc = std::max(3, 3 * c->sweep_depth);
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

    auto bail = [&](int rc) {
        g_create_error = c->err;
        iblb_destroy(c);
        return rc;
    };
    if (hipSetDevice(c->device) != hipSuccess) return bail(fail(c, IBLB_ERR_HIP, "hipSetDevice failed"));
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(c, IBLB_ERR_HIP, "hipStreamCreate failed"));

    // layout: g[xc*col + k*plane + y], the 9 planes of a column adjacent (plane = ny rounded up to
    // whole waves; col = 9 planes + 64 elements in f64: 4096^2 0.398 ms vs 0.425 ms with planes
    // apart, profiles/r01d_tune_layout_f64.log); gc ghost columns on each side; buffer 1 starts
    // 320 elements (f64) after the end of buffer 0 (profiles/r01_tune_f64_pads.log)
    const long rows = (long)round_up((size_t)c->ny, (size_t)(64 * c->V));
    c->L.ny = c->ny;
    c->L.ncol = c->ncol;
    c->L.rows = rows;
    c->L.plane = rows;
    c->L.col = 9 * rows + (f64 ? 64 : 0);
    const long width = (long)c->ncol + 2L * c->gc;
    c->fplane = width * rows;
    const long buf = width * c->L.col;
    const long gap = f64 ? 320 : 0;
    int rc;
    if ((rc = alloc_zero(c, (void**)&c->g_alloc, (size_t)(2 * buf + gap + 2 * GUARD) * c->esize))) return bail(rc);
    const long c0 = GUARD + (long)c->gc * c->L.col;  // column 0 of buffer 0
    c->g[0] = c->g_alloc + c0 * c->esize;
    c->g[1] = c->g_alloc + (c0 + buf + gap) * c->esize;
    c->buf_elems = buf;
    if ((rc = alloc_zero(c, (void**)&c->d_Q, 4 * sizeof(double)))) return bail(rc);
    if (c->max_points > 0) {
        const size_t np = (size_t)c->max_points;
        if ((rc = alloc_zero(c, (void**)&c->d_s, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_us, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_Fs, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_eps, np * sizeof(int)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->d_Fs_sum, 2 * np * sizeof(float)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->fd_alloc, 2 * (size_t)c->fplane * sizeof(double)))) return bail(rc);
        if ((rc = alloc_zero(c, (void**)&c->fl_alloc, (size_t)width * c->nch))) return bail(rc);
        c->fdense = c->fd_alloc + (long)c->gc * rows;
        c->flags = c->fl_alloc + (long)c->gc * c->nch;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(fail(c, IBLB_ERR_HIP, "allocation clear failed"));
    *out = c;
    return IBLB_OK;
}

void iblb_destroy(iblb_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    hold_release(c);  // (a test hold releases its kernel by itself)
    for (hipStream_t s : {c->stream, c->comm_stream})
        if (s) (void)hipStreamSynchronize(s);
    band_release(c);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    for (hipEvent_t e : {c->ev_bnd, c->ev_int, c->ev_int2, c->ev_pre, c->ev_x, c->ev_rccl})
        if (e) (void)hipEventDestroy(e);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    void* bufs[] = {c->g_alloc, c->cil_samples, c->cil_lasts, c->cil_bpoints, c->rho0, c->u0, c->force0, c->d_s,
                    c->d_us, c->d_Fs, c->d_eps, c->d_Fs_sum, c->fd_alloc, c->fl_alloc, c->d_Q, c->d_sch_s,
                    c->d_sch_us, c->d_sch_eps};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (c->sig) (void)hipFree(c->sig);
    if (c->sig_err) (void)hipHostFree(c->sig_err);
    if (c->hold_word) (void)hipHostFree(c->hold_word);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->left && c->left->right == c) c->left->right = nullptr;
    if (c->right && c->right->left == c) c->right->left = nullptr;
    delete c;
}

int iblb_set_state(iblb_ctx* c, const double* rho, const double* u, const double* f, const double* force) {
    if (!c) return IBLB_ERR_ARG;
    c->deep_chain = false;  // the state is rewritten: no deep cycle chain across this
    HIP_TRY(c, hipSetDevice(c->device));
    for (hipStream_t s : {c->stream, c->comm_stream, c->band_st, c->deep_st})
        if (s) HIP_TRY(c, hipStreamSynchronize(s));
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
    if (is_f64(c)) HIP_TRY(c, launch_pop_in<double>((const double*)d_f.p, gptr<double>(c, c->cur), c->L, c->stream));
    else HIP_TRY(c, launch_pop_in<float>((const double*)d_f.p, gptr<float>(c, c->cur), c->L, c->stream));
    HIP_TRY(c, launch_field_in((const double*)d_rho.p, c->rho0, c->L, 1, c->fplane, c->stream));
    HIP_TRY(c, launch_field_in((const double*)d_u.p, c->u0, c->L, 2, c->fplane, c->stream));
    HIP_TRY(c, launch_field_in((const double*)d_force.p, c->force0, c->L, 2, c->fplane, c->stream));
    HIP_TRY(c, hipMemsetAsync(c->d_Q, 0, 4 * sizeof(double), c->stream));
    if (c->fd_alloc) {
        HIP_TRY(c, hipMemsetAsync(c->fd_alloc, 0, 2 * (size_t)c->fplane * sizeof(double), c->stream));
        HIP_TRY(c, hipMemsetAsync(c->fl_alloc, 0, (size_t)(c->ncol + 2 * c->gc) * c->nch, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->cilia_on) {  // the beat restarts with the state (lasts = 0, main.cu:348-359)
        if ((rc = reset_cilia_state(c))) return rc;
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    c->phase = PH_BOOT;
    c->t = 0;
    c->ib_state = IB_NONE;
    c->ghost = 0;
    c->bnd_w = INT_MAX;
    return IBLB_OK;
}

int iblb_set_lagrangian(iblb_ctx* c, int ns, const float* s, const float* u_s, const int* epsilon) {
    if (!c || ns < 0) return IBLB_ERR_ARG;
    if (ns > c->max_points) return fail(c, IBLB_ERR_ARG, "ns exceeds max_points of the context");
    if (ns > 0 && (!s || !u_s)) return IBLB_ERR_ARG;
    if (c->cilia_on) return fail(c, IBLB_ERR_STATE, "cilia kinematics active: points come from iblb_set_cilia");
    int rc = check_slab_points(c, (size_t)ns, s);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = retire_points(c))) return rc;  // force^t still owed to the old points
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
    c->pts_host = ns > 0 ? host_points(s, (size_t)ns) : std::vector<float>();
    c->band_sticky = false;
    c->band_valid = false;
    c->band_dirty = ns > 0;  // planned at the next iblb_step (a slab needs its group)
    return IBLB_OK;
}

int iblb_set_lagrangian_steps(iblb_ctx* c, int nsteps, int ns, const float* s, const float* u_s, const int* epsilon) {
    if (!c || ns < 0 || nsteps < 1) return IBLB_ERR_ARG;
    if (ns > c->max_points) return fail(c, IBLB_ERR_ARG, "ns exceeds max_points of the context");
    if (ns > 0 && (!s || !u_s)) return IBLB_ERR_ARG;
    if (c->cilia_on) return fail(c, IBLB_ERR_STATE, "cilia kinematics active: points come from iblb_set_cilia");
    const size_t np = (size_t)nsteps * ns;
    int rc = check_slab_points(c, np, s);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = retire_points(c))) return rc;  // the force owed to the points before the schedule
    // host copies for the per-cycle band plans: every entry's (x, y), and the points before the
    // schedule (a force evaluated from them is owed to the first iteration)
    c->sch_x_prev.clear();
    if (c->ns > 0 && c->ib_state == IB_READY) c->sch_x_prev = c->pts_host;
    if (ns > 0) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if ((rc = sched_reserve(c, (size_t)nsteps, ns))) return rc;
        HIP_TRY(c, hipMemcpyAsync(c->d_sch_s, s, 2 * np * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(c->d_sch_us, u_s, 2 * np * sizeof(float), hipMemcpyHostToDevice, c->stream));
        if (epsilon) {
            HIP_TRY(c, hipMemcpyAsync(c->d_sch_eps, epsilon, np * sizeof(int), hipMemcpyHostToDevice, c->stream));
        } else {
            std::vector<int> ones(np, 1);
            HIP_TRY(c, hipMemcpyAsync(c->d_sch_eps, ones.data(), np * sizeof(int), hipMemcpyHostToDevice, c->stream));
        }
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->sch_x = host_points(s, np);
    }
    c->ns = ns;
    c->sch_t0 = c->t;
    c->sch_n = ns > 0 ? nsteps : 0;
    c->sch_cur = -1;  // d_s holds the points before the schedule (retire_points)
    c->band_sticky = true;
    c->band_valid = false;  // planned per cycle (plan_cycle)
    c->band_retry_t = 0;
    c->band_dirty = false;
    return IBLB_OK;
}

int iblb_set_cilia(iblb_ctx* c, const iblb_cilia* k) {
    if (!c) return IBLB_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc;
    if (c->phase == PH_RUN || c->ib_state == IB_PENDING) {
        if ((rc = retire_points(c))) return rc;  // force still owed to the current points
    }
    c->band_valid = false;  // the points now come from the kinematics
    c->band_dirty = false;
    c->sch_n = 0;
    c->sch_cur = -1;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (float* p : {c->cil_samples, c->cil_lasts, c->cil_bpoints})
        if (p) (void)hipFree(p);
    c->cil_samples = c->cil_lasts = c->cil_bpoints = nullptr;
    c->cilia_on = false;
    if (!k || k->c_num <= 0) return IBLB_OK;
    if (k->T <= 0 || !(k->c_space > 0)) return fail(c, IBLB_ERR_ARG, "cilia: need T > 0 and c_space > 0");
    if (CILIA_POINTS * k->c_num > c->max_points) return fail(c, IBLB_ERR_ARG, "cilia: max_points must be >= 96 * c_num");
    c->cilia = *k;
    const size_t nk = (size_t)CILIA_SAMPLES * k->c_num;
    HIP_TRY(c, hipMalloc(&c->cil_samples, 5 * nk * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->cil_lasts, 2 * nk * sizeof(float)));
    HIP_TRY(c, hipMalloc(&c->cil_bpoints, 5 * (size_t)CILIA_POINTS * k->c_num * sizeof(float)));
    if ((rc = reset_cilia_state(c))) return rc;
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
    if (is_f64(c))
        HIP_TRY(c, launch_pop_out<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), (double*)df.p, raw,
                                          c->stream));
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
        if ((rc = rccl_order(c, c->stream))) return rc;
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
        if (is_f64(c))
            HIP_TRY(c, launch_flux<double>(gptr<double>(c, c->cur), c->L, halo_of<double>(c, c->cur), fd, c->fplane,
                                           c->coef.gx, c->coef.gy, fc, c->cfg.flux_norm, c->d_Q + 1, c->stream));
        else
            HIP_TRY(c, launch_flux<float>(gptr<float>(c, c->cur), c->L, halo_of<float>(c, c->cur), fd, c->fplane,
                                          c->coef.gx, c->coef.gy, fc, c->cfg.flux_norm, c->d_Q + 1, c->stream));
    }
    if (rccl_multi(c)) {
        if ((rc = rccl_order(c, c->stream))) return rc;
        NCCL_TRY(c, ncclAllReduce(c->d_Q + 1, c->d_Q + 1, 1, ncclFloat64, ncclSum, c->comm, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(Q, c->d_Q + 1, sizeof(double), hipMemcpyDeviceToHost));
    return IBLB_OK;
}

int iblb_count_nonfinite(iblb_ctx* c, long long* count) {
    if (!c || !count) return IBLB_ERR_ARG;
    int rc = check_ready(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = band_join(c)) || (rc = join_comm(c))) return rc;
    HIP_TRY(c, hipMemsetAsync(c->d_Q + 1, 0, sizeof(double), c->stream));
    if (is_f64(c)) HIP_TRY(c, launch_count_nonfinite<double>(gptr<double>(c, c->cur), c->L, c->d_Q + 1, c->stream));
    else HIP_TRY(c, launch_count_nonfinite<float>(gptr<float>(c, c->cur), c->L, c->d_Q + 1, c->stream));
    if (rccl_multi(c)) {
        if ((rc = rccl_order(c, c->stream))) return rc;
        NCCL_TRY(c, ncclAllReduce(c->d_Q + 1, c->d_Q + 1, 1, ncclFloat64, ncclSum, c->comm, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    double n = 0.;
    HIP_TRY(c, hipMemcpy(&n, c->d_Q + 1, sizeof(double), hipMemcpyDeviceToHost));
    *count = (long long)n;
    return IBLB_OK;
}

int iblb_get_step(iblb_ctx* c, long long* steps) {
    if (!c || !steps) return IBLB_ERR_ARG;
    *steps = c->t;
    return IBLB_OK;
}

int iblb_set_profiling(iblb_ctx* c, int enabled) {
    if (!c) return IBLB_ERR_ARG;
    c->prof = enabled == 2 ? 2 : enabled != 0 ? 1 : 0;
    return IBLB_OK;
}

int iblb_get_timing(iblb_ctx* c, iblb_timing* t, int reset) { return iblb_get_timing_ex(c, t, sizeof(*t), reset); }

int iblb_get_timing_ex(iblb_ctx* c, iblb_timing* out, unsigned long bytes, int reset) {
    if (!c || !out || bytes == 0) return IBLB_ERR_ARG;
    iblb_timing full{};
    iblb_timing* t = &full;
    HIP_TRY(c, hipSetDevice(c->device));
    for (hipStream_t s : {c->stream, c->comm_stream, c->band_st, c->deep_st})
        if (s) HIP_TRY(c, hipStreamSynchronize(s));
    int rc = ev_drain(c);
    if (rc) return rc;
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
    t->band_cycles = c->band_cycles;
    t->band_merged_cycles = c->band_merged_cycles;
    t->band_par_cycles = c->band_par_cycles;
    t->deep_launches = c->deep_launches;
    t->deep_iterations = c->deep_iterations;
    t->dev_wait_launches = c->dev_wait_launches;
    t->deep_mode = c->deep_kinfo[0];
    t->deep_vs = c->deep_kinfo[1];
    t->deep_waves_per_simd = c->deep_kinfo[2];
    t->deep_vgprs = c->deep_kinfo[3];
    if (reset) {
        c->band_cycles = c->band_merged_cycles = c->band_par_cycles = 0;
        c->deep_launches = c->deep_iterations = 0;
        c->dev_wait_launches = 0;
        c->fused_ms = c->ib_ms = c->halo_ms = c->sweep_ms = c->sweepk_ms = 0.;
        c->fused_launches = c->fused_cells = c->sweep_launches = c->sweep_cells = 0;
        c->sweepk_launches = c->sweepk_cells = 0;
    }
    std::memcpy(out, &full, std::min((size_t)bytes, sizeof(full)));
    return IBLB_OK;
}

int iblb_get_stream(iblb_ctx* c, void** stream) {
    if (!c || !stream) return IBLB_ERR_ARG;
    *stream = (void*)c->stream;
    return IBLB_OK;
}

int iblb_set_wait_timeout(iblb_ctx* c, double seconds) {
    if (!c || !(seconds > 0.)) return IBLB_ERR_ARG;
    c->wait_timeout_s = seconds;
    if (c->clock_hz <= 0.) return IBLB_OK;  // (the ticks are derived at the RCCL attach)
    HIP_TRY(c, hipSetDevice(c->device));
    return set_wait_ticks(c);
}

int iblb_synchronize(iblb_ctx* c) {
    if (!c) return IBLB_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    for (hipStream_t s : {c->stream, c->comm_stream, c->band_st, c->deep_st})
        if (s) HIP_TRY(c, hipStreamSynchronize(s));
    return check_wait_err(c);
}

// ---- output gather (RCCL group) -----------------------------------------------------------------
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
    if ((rc = rccl_order(c, c->stream))) return rc;
    // rank r's [rho | u] block lands at 3*ny*x_begin_r in rank order
    NCCL_TRY(c, ncclGroupStart());
    if (is_root) {
        for (int r = 0; r < c->nranks; ++r) {
            double* dst = (double*)all.p + 3L * c->ny * c->slab_begin[r];
            const size_t n = 3 * (size_t)c->ny * c->slab_count[r];
            if (r == root) HIP_TRY(c, hipMemcpyAsync(dst, mine.p, n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
            else NCCL_TRY(c, ncclRecv(dst, n, ncclFloat64, r, c->comm, c->stream));
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

}  // extern "C"

// ---- checkpoint / restart -------------------------------------------------------------------------
// File: 8-byte magic, 12 int64 fields, 6 doubles, then the stored populations g (plane i, column
// xc, rows y; storage precision, no padding), the Lagrangian points and the cilia buffers.
namespace {
const char CKPT_MAGIC[8] = {'I', 'B', 'L', 'B', 'C', 'K', '0', '1'};
enum { CK_VERSION, CK_NX, CK_NY, CK_XB, CK_NCOL, CK_PREC, CK_T, CK_NS, CK_CILIA, CK_CNUM, CK_CT, CK_CPSTEP, CK_NI };
enum { CK_Q, CK_CSPACE, CK_TAU, CK_TAU2, CK_GX, CK_GY, CK_ND };

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) std::fclose(f);
    }
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

extern "C" {

int iblb_save_checkpoint(iblb_ctx* c, const char* path) {
    if (!c || !path) return IBLB_ERR_ARG;
    if (c->phase != PH_RUN) return fail(c, IBLB_ERR_STATE, "checkpoint needs a state advanced by at least one step");
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = iblb_synchronize(c);
    if (rc) return rc;
    File fl;
    const std::string tmp = std::string(path) + ".tmp";
    fl.f = std::fopen(tmp.c_str(), "wb");
    if (!fl.f) return fail(c, IBLB_ERR_ARG, std::string("cannot open ") + tmp + " for writing");
    double Q = 0.;
    HIP_TRY(c, hipMemcpy(&Q, c->d_Q, sizeof(double), hipMemcpyDeviceToHost));
    long long iv[CK_NI] = {1, c->nx, c->ny, c->x_begin, c->ncol, c->prec, c->t, c->ns, c->cilia_on ? 1 : 0,
                           c->cilia.c_num, c->cilia.T, c->cilia.p_step};
    double dv[CK_ND] = {Q, c->cilia.c_space, c->cfg.tau, c->cfg.tau2, c->coef.gx, c->coef.gy};
    rc = ck_io(c, std::fwrite(CKPT_MAGIC, 1, 8, fl.f) == 8 && std::fwrite(iv, sizeof(iv), 1, fl.f) == 1 &&
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
    int rc = iblb_synchronize(c);
    if (rc) return rc;
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
    // cilia configuration first (allocates its buffers), then every array
    c->ib_state = IB_NONE;
    c->phase = PH_EMPTY;
    if (iv[CK_CILIA]) {
        iblb_cilia k{(int)iv[CK_CNUM], dv[CK_CSPACE], (int)iv[CK_CT], (int)iv[CK_CPSTEP]};
        if ((rc = iblb_set_cilia(c, &k))) return rc;
    } else if (c->cilia_on) {
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
    if (c->fd_alloc) {
        HIP_TRY(c, hipMemsetAsync(c->fd_alloc, 0, 2 * (size_t)c->fplane * sizeof(double), c->stream));
        HIP_TRY(c, hipMemsetAsync(c->fl_alloc, 0, (size_t)(c->ncol + 2 * c->gc) * c->nch, c->stream));
    }
    c->ns = (int)ns;
    c->sch_n = 0;  // the restored points are static
    c->sch_cur = -1;
    c->band_sticky = false;
    c->band_valid = false;
    c->band_retry_t = 0;
    c->pts_host.clear();
    if (ns > 0 && !c->cilia_on) {  // host copy for the band plan of the restored points
        c->pts_host.resize(2 * ns);
        HIP_TRY(c, hipMemcpy(c->pts_host.data(), c->d_s, c->pts_host.size() * sizeof(float), hipMemcpyDeviceToHost));
    }
    c->band_dirty = ns > 0 && !c->cilia_on;
    c->t = iv[CK_T];
    c->phase = PH_RUN;
    c->ghost = 0;
    c->bnd_w = INT_MAX;
    c->ib_state = ib_active(c) ? IB_PENDING : IB_NONE;  // force^t is re-evaluated from g and the points
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return IBLB_OK;
}

}  // extern "C"
