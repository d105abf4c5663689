// ctx_band.hip — the IB band cycle: K iterations per cycle with an owed IB force every iteration.
//
// The force of iteration t+j is nonzero only in the forced cells of the points (columns x0-1 ..
// x0+1, rows y0-1 .. y0+1), and after K iterations a cell depends only on forces within K-1 cells
// of it.  So a cycle splits the lattice:
//  * patches — the forced cells of every point the cycle sees (static points, or the K entries of a
//    schedule given ahead with iblb_set_lagrangian_steps), merged into column intervals with their
//    row range; a patch's output is its columns +- (K-1) and rows +- (K-1);
//  * the trapezoid of a patch: level j = 0 .. K-1 over the output +- (K-1-j) more columns and rows
//    (R = 2(K-1) columns beyond the forced ones at level 0), g^t -> scratch -> ... -> g^{t+K}, one
//    one-step launch per level over the (column, row chunk) entries of all patches, with the IB
//    kernel evaluating force^{t+j} from level j-1 — with the points of iteration t+j-1 — before
//    level j; the last level stores the patch output rows of the slab's own columns;
//  * the deep sweep — one sweepk launch over every column (a slab of a group: its interior, the
//    boundary sweeps on the comm stream doing [0, K) and [ncol-K, ncol)); it ignores the force, so
//    its output is exact outside the patches' outputs, which the trapezoid's last level overwrites
//    after it.  The flux column's patch rows are skipped by the deep sweeps (fskip) and added by the
//    trapezoid, every level.
// Every cell of g^{t+K} is written last by the same code as a one-step iteration would run, so the
// result equals K one-step iterations (up to the arrival order of the spread atomics).
//
// Patches near or across a slab edge (round 3).  A trapezoid whose level-0 input leaves the slab
// reads its ghost columns: a slab of a group receives gc = 3K of them from each neighbour (one
// exchange per cycle, the same depth on every rank), a lone slab fills them with periodic copies
// of its own edge columns.  The trapezoid then advances the ghost columns too — redundantly, from
// the same data as the neighbour — with the points' periodic images (ib_ghost_group), clipped at
// the ghost edge; the garbage that enters there (pulls beyond the ghosts) travels at most 3
// columns per level (a force's nodes reach 2, their pulls 3), so after K levels it stops short of
// the slab's own columns when gc >= 3K.  Only the slab's own columns are stored.
#include <cmath>
#include <cstdio>
#include <cstring>

#include <functional>

#include "ctx.h"

namespace iblbh {

// a slab of an RCCL group: the cycle's halo exchange and boundary sweeps need the comm stream and
// slabs of >= 4K columns (and >= gc: the ghosts are whole columns of the neighbour); every rank
// takes the same decision (the narrowest slab of the group)
static bool band_slab_ok(const iblb_ctx* c) {
    const int K = c->sweep_depth;
    return rccl_multi(c) && c->overlap && c->comm_stream && c->min_slab >= std::max(4 * K, c->gc);
}

bool band_ready(const iblb_ctx* c) {
    return c->band_on && c->band_valid && (single_slab(c) || band_slab_ok(c)) && c->phase == PH_RUN &&
           (!c->cilia_on || c->cil_sched) && ib_active(c) && c->sweep_on && c->sweep_depth >= 3;
}

bool band_possible(const iblb_ctx* c) {
    return c->band_on && c->sweep_on && c->sweep_depth >= 3 && c->phase != PH_EMPTY &&
           (single_slab(c) || band_slab_ok(c));
}

// Streams of the overlapped band cycle: the band chain on band_st restricted to `band_reserve` CUs
// (the top mask bits of the CUs the cycle may use: bit i is a CU of XCD i % 8, so 8m bits are m CUs
// of every XCD, profiles/r02n_xcc_probe.txt), the cycle's deep sweep on deep_st masked to the
// others.  A lone slab may use the whole chip; a slab of an RCCL group the compute stream's CUs
// (the comm stream keeps its reserved CUs for the exchange and the boundary sweeps).  The context's
// stream is never replaced: both start after it and it waits for both.  The chain (2K dependent
// small launches, latency-bound: ~8 us each uncontended) gets one XCD's worth of CUs, two where the
// trapezoids hold more than 5 % of the cycle's lattice updates.  A lone slab whose deep sweep runs
// for at least 1.5x that chain (>= 4M cells a level at K = 5, 2048^2 and up) instead leaves both
// streams unmasked with the chain's at the highest priority: the chain has the slack to wait for CUs
// the deep sweep's workgroups free, and the deep sweep gets the whole chip (profiles/r03ch: K3 +5 %,
// K5 +5 %; the K5-width slab 1024 x 2048, whose chain is as long as its deep sweep, -4 to -9 %).
static int band_streams(iblb_ctx* c, long long band_cols, long long deep_cols) {
    const bool slab = rccl_multi(c);
    int rc_;
    if (c->transport == TR_LOCAL) return IBLB_OK;
    if (!c->ncu) {
        hipDeviceProp_t prop;
        HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
        c->ncu = prop.multiProcessorCount;
    }
    const int per_xcd = std::max(1, c->ncu / 8);
    const double share = (double)band_cols / (double)std::max(1LL, band_cols + (long long)c->sweep_depth * deep_cols);
    long want = (share > 0.05 ? 2 : 1) * per_xcd;
    const double deep_us = (double)c->sweep_depth * deep_cols * c->ny / (is_f64(c) ? 130e3 : 190e3);
    // a group slab's merged chain at depth >= 7 (its short deep sweep, plan_bands_t): two XCDs' worth.
    // Its launches (~640 waves on the K5-width slab) take two rounds on 32 CUs at four waves per SIMD;
    // self ring, five alternations (profiles/r04/cus3264): 2048 x 2048 edge 0.0320 vs 0.0342 ms per
    // iteration, 1024 x 2048 edge 0.0242 vs 0.0250, mid-slab equal; the chained chain beside the long
    // deep sweep of a 4096-column slab keeps one (0.0495 vs 0.0546 with two, profiles/r04/slabcus)
    const bool merged = c->band_merge == 2 || (c->band_merge == 1 && deep_us < 1.5 * 2 * c->sweep_depth * 8.0);
    if (slab && merged && c->sweep_depth >= 7) want = 2 * per_xcd;
    // f32 at depth >= 7: the chain on one XCD's worth of CUs of its own and the deep sweep in its own
    // build (the packed wall split) on the rest: K5 242.5-243.2k MLUPS against 221.4-221.9k for both
    // streams unmasked beside the scalar build, 231.5-232.7k unmasked beside the packed split; the
    // chain on 16 / 64 CUs 178k / 212k (profiles/r04/k5var).  (At depth 5 the same arrangement lost:
    // 196-207k vs 221-227k, profiles/r04/k5deep.)  f64: both unmasked (K3 136k vs 128k masked).
    bool own_build = false;
    if (!slab && deep_us >= 1.5 * 2 * c->sweep_depth * 8.0) {
        if (!is_f64(c) && c->sweep_depth >= 7) {
            want = per_xcd;
            own_build = true;
        } else {
            want = -2;
        }
    }
    std::vector<uint32_t> base((size_t)(c->ncu + 31) / 32, 0u);
    int avail = 0;
    for (int i = 0; i < c->ncu; ++i)
        if (!slab || c->comp_mask.empty() || (c->comp_mask[(size_t)i / 32] >> (i % 32) & 1u)) {
            base[(size_t)i / 32] |= 1u << (i % 32);
            ++avail;
        }
    // IBLB_BAND_CUS: CUs of the chain's stream; -2: both streams unmasked, the chain's at the highest
    // priority; 0: one stream, the chain and the deep sweep in sequence
    want = env_long("IBLB_BAND_CUS", want);
    if (want == -2 && slab) want = per_xcd;  // a group slab's comm stream owns the reserved CUs
    if (want >= avail) want = 0;
    c->band_own_build = own_build && want > 0;  // (the chain masked to CUs of its own, any count: IBLB_BAND_CUS)
    if (want == c->band_reserve || (c->band_sticky && c->band_st)) return IBLB_OK;
    if ((rc_ = band_join(c))) return rc_;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (hipStream_t* st : {&c->band_st, &c->deep_st})
        if (*st) {
            HIP_TRY(c, hipStreamSynchronize(*st));
            (void)hipStreamDestroy(*st);
            *st = nullptr;
        }
    if (want == -2) {
        int lo = 0, hi = 0;
        HIP_TRY(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(c, hipStreamCreateWithPriority(&c->band_st, hipStreamNonBlocking, hi));
        HIP_TRY(c, hipStreamCreateWithFlags(&c->deep_st, hipStreamNonBlocking));
    } else if (want > 0) {
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
    }
    for (hipEvent_t* e : {&c->ev_b0, &c->ev_bd, &c->ev_deep})
        if (!*e) HIP_TRY(c, hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventDisableSystemFence));
    c->band_reserve = (int)want;
    return IBLB_OK;
}

// periodic distance from global column f to the nearest slab edge of the group
static int edge_distance(const iblb_ctx* c, int f) {
    int best = INT_MAX;
    for (int e : c->slab_begin) {
        int d = std::abs(f - e) % c->nx;
        best = std::min(best, std::min(d, c->nx - d));
    }
    return best;
}

// Band plan for band_step from the (x, y) of every point the cycle may see (host copy: the static
// points, or the cycle's schedule entries plus the point before them).  band_valid stays false
// where the cycle does not apply or does not pay (a lone slab's trapezoids over half the lattice).
template <typename T>
static int plan_bands_t(iblb_ctx* c, const std::vector<float>& xy) {
    const int K = c->sweep_depth, R = 2 * (K - 1);
    const bool slab = !single_slab(c);
    const int ncol = c->ncol, ny = c->ny, nx = c->nx, D = c->gc;
    const int lo = -D + 1, hi = ncol + D - 2;  // level-0 columns a trapezoid may cover (local)
    const int W = ncol + 2 * D;
    // forced cells of every point image in [lo, hi]: a row range per local column (index x + D);
    // and whether any point forces a column near any slab edge (the group's exchange depth: every
    // rank holds every point, so every rank finds the same answer)
    std::vector<int> fy0((size_t)W, INT_MAX), fy1((size_t)W, INT_MIN);
    const int zone = std::max(D, R + 2);
    bool edge_any = false;
    // consecutive points in one column (a filament's) accumulate their rows in registers and update
    // the column table once: per-point updates of the same few entries chain through store-to-load
    // forwarding (768 points x K+1 iterations: 131 -> 24 us per plan on a container core)
    int cx = INT_MIN, cy0 = 0, cy1 = 0;
    auto flush = [&]() {
        if (cx == INT_MIN) return;
        for (int dx = -1; dx <= 1; ++dx) {
            const int xg = cx + dx;  // forced global column (the spread has no periodic image)
            if (xg < 0 || xg >= nx) continue;
            if (slab && !edge_any && edge_distance(c, xg) <= zone) edge_any = true;
            for (int m = -1; m <= 1; ++m) {
                const int x = xg - c->x_begin + m * nx;
                if (x < lo || x > hi) continue;
                fy0[(size_t)(x + D)] = std::min(fy0[(size_t)(x + D)], cy0);
                fy1[(size_t)(x + D)] = std::max(fy1[(size_t)(x + D)], cy1);
            }
        }
    };
    for (size_t k = 0; k + 1 < xy.size(); k += 2) {
        const int x0 = (int)std::nearbyint((double)xy[k]);
        const int y0 = (int)std::nearbyint((double)xy[k + 1]);
        const int ya = std::min(std::max(0, y0 - 1), ny - 1), yb = std::max(std::min(ny - 1, y0 + 1), 0);
        if (x0 == cx) {
            cy0 = std::min(cy0, std::min(ya, yb));
            cy1 = std::max(cy1, std::max(ya, yb));
            continue;
        }
        flush();
        cx = x0;
        cy0 = std::min(ya, yb);
        cy1 = std::max(ya, yb);
    }
    flush();
    // forced column intervals with their row range, merged into patches {x0, x1, y0, y1} whose
    // trapezoids stay apart (gaps >= 2R + 8 columns)
    std::vector<std::array<int, 4>> b;
    for (int x = lo; x <= hi;) {
        if (fy0[(size_t)(x + D)] > fy1[(size_t)(x + D)]) { ++x; continue; }
        std::array<int, 4> iv{x, x, fy0[(size_t)(x + D)], fy1[(size_t)(x + D)]};
        while (iv[1] + 1 <= hi && fy0[(size_t)(iv[1] + 1 + D)] <= fy1[(size_t)(iv[1] + 1 + D)]) {
            ++iv[1];
            iv[2] = std::min(iv[2], fy0[(size_t)(iv[1] + D)]);
            iv[3] = std::max(iv[3], fy1[(size_t)(iv[1] + D)]);
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
    // ghosts: a trapezoid whose level-0 input [x0 - R - 1, x1 + R + 1] leaves the slab reads D
    // ghost columns (and the garbage frontier argument above needs all of them)
    bool need = false;
    for (auto& p : b) need |= p[0] - R - 1 < 0 || p[1] + R + 1 > ncol - 1;
    const int bd = need ? D : 0;
    const int bx = slab ? std::max(K, edge_any ? D : 0) : 0;
    if (need && (slab ? !edge_any : ncol < D)) {  // (cannot happen for a slab: need implies edge_any)
        c->band_valid = false;
        return IBLB_OK;
    }
    if (c->band_valid && b == c->band_b && bd == c->band_d && bx == c->band_x) return IBLB_OK;
    c->band_valid = false;
    // Rows: a patch's output rows [ya, yb) = its forced rows +- (K-1); level j covers K-1-j more on
    // each side (the deep sweep advances every row, the last level overwrites the output rows)
    // (even bounds: a lane of the deep sweep's two-cell walk is then wholly in or out of a patch
    // output, which the deep sweep leaves to the last level when the two run side by side)
    // the chain's flavour first (the level launches' row chunks depend on it): merged chain (IBLB_BAND_MERGE
    // 1 = auto) where the chain, not the deep sweep beside it, is the cycle's critical path (the deep sweep
    // shorter than 1.5x a chain of 2K ~8 us launches: narrow slabs).  Its launches are longer than the
    // one-step launches they replace (the point groups recompute the level's collide over their nodes'
    // pulls): beside a long deep sweep it only adds work (K3 0.0378 vs 0.0359 ms/iteration); on the
    // K5-width slab it saves 3-6 % (profiles/r03mg)
    const long long deep_cols = slab ? std::max(0, ncol - 2 * K) : ncol;  // the deep sweep's columns
    {
        const double deep_us = (double)K * deep_cols * ny / (is_f64(c) ? 130e3 : 190e3);
        c->band_merged = c->band_merge == 2 || (c->band_merge == 1 && deep_us < 1.5 * 2 * K * 8.0);
    }
    // Half-height level waves (f32, IBLB_BAND_VHALF, round 6): a level launch's entry waves take
    // 64 * V/2 rows (two cells per lane) instead of 64 * V: a patch's row range (K5's filaments: ~110
    // rows) then spans fewer padding rows than in 256-row chunks, and the chain — K5's critical path
    // beside the deep sweep (profiles/r06/k5tl) — computes fewer cells
    c->band_vhalf = !is_f64(c) && c->band_vhalf_env != 0;
    const int V64 = 64 * (c->band_vhalf ? c->V / 2 : c->V);  // rows per chunk of the level launches
    const int nchv = (ny + V64 - 1) / V64;                     // such chunks per column
    std::vector<std::array<int, 2>> pr(b.size());
    for (size_t q = 0; q < b.size(); ++q)
        pr[q] = {std::max(0, b[q][2] - (K - 1)) & ~1, std::min(ny, (b[q][3] + K + 1) & ~1)};
    std::vector<int> tab;
    std::vector<int> off((size_t)K), cnt((size_t)K), nchl((size_t)K, 0);
    long long band_lu = 0;
    for (int j = 0; j < K; ++j) {
        off[j] = (int)tab.size();
        cnt[j] = 0;
        const int m = K - 1 - j;
        const int lj = -bd + 1 + j, hj = ncol + bd - 2 - j;  // columns level j can compute
        for (size_t q = 0; q < b.size(); ++q) {
            const int ylo = std::max(0, pr[q][0] - m), yhi = std::min(ny, pr[q][1] + m);
            const int ch0 = ylo / V64, ch1 = std::min(nchv, (yhi + V64 - 1) / V64);
            int xa = std::max(b[q][0] - R + j, lj), xb = std::min(b[q][1] + R - j, hj);
            if (j == K - 1) {  // the last level stores the slab's own columns only
                xa = std::max(xa, 0);
                xb = std::min(xb, ncol - 1);
            }
            if (xa > xb) continue;
            nchl[j] = std::max(nchl[j], ch1 - ch0);
            for (int x = xa; x <= xb; ++x) {
                tab.insert(tab.end(), {x, ch0, ch1, pr[q][0], pr[q][1]});
                ++cnt[j];
                band_lu += std::min(ny, ch1 * V64) - ch0 * V64;
            }
        }
    }
    if (!slab && 2 * band_lu > (long long)K * nx * ny) return IBLB_OK;
    // the deep sweep: every column of a lone slab, the interior [K, ncol-K) of a group slab (deep_cols)
    int rc = band_streams(c, band_lu / std::max(1, ny), deep_cols);
    if (rc) return rc;
    // the tables go to a ring of pinned (device-visible, coherent) host slots that the cycle's
    // launches read directly: a new plan of moving points costs no copy on the cycle's critical
    // path; a slot is rewritten only after the event of the last cycle that read it.  (Round 6 tried a
    // device copy of each new plan's slot on the chain's stream: K5, whose moving points bring a new plan
    // every cycle, 0.52-0.62 ms per cycle against 0.441-0.445; K3's static plan equal, profiles/r06/dt1)
    if (tab.size() > c->band_pin_cap) {  // every slot may be in use: wait for the cycles in flight
        if ((rc = band_join(c))) return rc;
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        const size_t cap = std::max(tab.size(), (size_t)5 * (K + 1) * (ncol + 2 * D) + 64);
        for (int i = 0; i < BAND_PIN_SLOTS; ++i) {
            if (c->band_pin[i]) (void)hipHostFree(c->band_pin[i]);
            c->band_pin[i] = nullptr;
        }
        c->band_pin_cap = 0;
        for (int i = 0; i < BAND_PIN_SLOTS; ++i)
            HIP_TRY(c, hipHostMalloc((void**)&c->band_pin[i], cap * sizeof(int), hipHostMallocCoherent));
        c->band_pin_cap = cap;
    }
    const int slot = c->band_pin_i;
    c->band_pin_i = (slot + 1) % BAND_PIN_SLOTS;
    if (c->band_pin_ev[slot]) HIP_TRY(c, hipEventSynchronize(c->band_pin_ev[slot]));
    else HIP_TRY(c, hipEventCreateWithFlags(&c->band_pin_ev[slot], hipEventDisableTiming));
    if (!tab.empty()) std::memcpy(c->band_pin[slot], tab.data(), tab.size() * sizeof(int));
    c->band_tab = c->band_pin[slot];
    c->band_pin_cur = slot;
    if (c->band_merged && !c->bf_alloc) {  // merged chain: the force buffers of levels j % 3 = 1, 2
        const size_t width = (size_t)c->ncol + 2 * c->gc;
        if ((rc = alloc_zero(c, (void**)&c->bf_alloc, 4 * (size_t)c->fplane * sizeof(double)))) return rc;
        if ((rc = alloc_zero(c, (void**)&c->bfl_alloc, 2 * width * c->nch))) return rc;
        for (int i = 0; i < 2; ++i) {
            c->bfd[i] = c->bf_alloc + (size_t)i * 2 * c->fplane + (long)c->gc * c->L.rows;
            c->bfl[i] = c->bfl_alloc + (size_t)i * width * c->nch + (long)c->gc * c->nch;
        }
    }
    if (!c->s_alloc) {  // the trapezoid's scratch levels: two buffers laid out like g
        const size_t bytes = (size_t)(2 * c->buf_elems + 2 * GUARD) * c->esize;
        if ((rc = alloc_zero(c, (void**)&c->s_alloc, bytes))) return rc;
        const long c0 = GUARD + (long)c->gc * c->L.col;  // column 0 of buffer 0
        c->sbuf[0] = c->s_alloc + c0 * c->esize;
        c->sbuf[1] = c->s_alloc + (c0 + c->buf_elems) * c->esize;
    }
    c->band_off = off;
    c->band_n = cnt;
    c->band_nchl = nchl;
    c->band_deep_lu = deep_cols * ny;
    c->band_lu = band_lu;
    c->band_flux = -1;
    c->band_fy0 = c->band_fy1 = 0;
    const int fc = c->cfg.flux_column - c->x_begin;
    if (fc >= 0 && fc < ncol)
        for (size_t q = 0; q < b.size(); ++q)
            if (fc >= b[q][0] - (K - 1) && fc <= b[q][1] + (K - 1)) {
                c->band_flux = fc;
                c->band_fy0 = pr[q][0];
                c->band_fy1 = pr[q][1];
            }
    c->band_b = b;
    c->band_d = bd;
    c->band_x = bx;
    // PAR (two streams): the last level beside the deep sweep (and a group slab's boundary sweeps),
    // which skip the patch outputs — the last level's entries: own columns [x0 - (K-1), x1 + (K-1)],
    // rows pr.  Only where those regions stay disjoint in columns (periodic images of a tiny slab
    // could overlap) and fit the kernel arguments.
    // IBLB_BAND_PAR 1 (auto): where the chain, not the deep sweep, is the cycle's critical path (the
    // merged chain's criterion: narrow slabs) — the deep sweep's per-column skip test costs it 9-14 %
    // (K3 114k vs 118k, K5 193k vs 218k MLUPS with it, profiles/r04/par); 2: always; 0: never
    c->band_skip.clear();
    c->band_par = false;
    const double deep_us = (double)K * deep_cols * ny / (is_f64(c) ? 130e3 : 190e3);
    if (c->band_st && (c->band_par_env == 2 || (c->band_par_env == 1 && deep_us < 1.5 * 2 * K * 8.0))) {
        bool ok = b.size() <= (size_t)MAX_SKIP;
        for (size_t q = 0; ok && q < b.size(); ++q) {
            const int x0 = std::max(0, b[q][0] - (K - 1)), x1 = std::min(ncol - 1, b[q][1] + (K - 1));
            if (x0 > x1) continue;
            if (!c->band_skip.empty() && x0 <= c->band_skip.back().x1) ok = false;
            c->band_skip.push_back(SkipBox{x0, x1, pr[q][0], pr[q][1]});
        }
        c->band_par = ok && !c->band_skip.empty();
        if (!c->band_par) c->band_skip.clear();
    }
    c->band_valid = true;
    return IBLB_OK;
}

int plan_bands(iblb_ctx* c, const std::vector<float>& xy) {
    c->band_dirty = false;
    if (!c->band_on || xy.empty() || c->sweep_depth < 3 || !c->sweep_on || (c->cilia_on && !c->cil_sched) ||
        !(single_slab(c) || band_slab_ok(c))) {
        c->band_valid = false;
        return IBLB_OK;
    }
    return is_f64(c) ? plan_bands_t<double>(c, xy) : plan_bands_t<float>(c, xy);
}

// The band plan of the cycle starting at iteration c->t under a schedule: the forces of its K
// levels come from the points of iterations t-1 .. t+K-2 (the force owed at the start was, or will
// be, evaluated from iteration t-1's points: the points before the schedule if t = t0).
int plan_cycle(iblb_ctx* c) {
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

// the cycle's deep sweep: every column of a lone slab, the interior [K, ncol-K) of a group slab;
// the rows of the flux column a patch accounts for are not sampled
template <typename T>
static int band_deep(iblb_ctx* c, int K, hipStream_t ds) {
    const bool slab = !single_slab(c);
    const int lo = slab ? K : 0, hi = slab ? c->ncol - K : c->ncol, n = hi - lo;
    if (n <= 0) return IBLB_OK;
    const int W = std::max(1, c->deep_w);
    Sweep2Args<T> d = sweep_args<T>(c, lo, c->deep_balance ? 0 : W, hi, (n + W - 1) / W, W);
    d.vs = slab ? c->slab_vs : c->deep_vs;
    // f32: the two-wave scalar-collide build: the three-wave f32 wall split leaves the chain's kernels
    // no room beside the deep sweep (K5 197.6k vs 193.9k MLUPS with it, profiles/r03sp), and the
    // packed builds (two waves of 191 / 228 VGPRs) measured 209k / 202k vs 215k (profiles/r04/pack)
    // -- except where the chain has CUs of its own beside a long deep sweep (band_own_build, depth
    // >= 7: K5 243k vs 222k MLUPS, profiles/r04/k5var).
    // f64: the configured variant (its wall split keeps one wave per SIMD; not with PAR's skip boxes)
    // without the LDS window (bit 7): its 144 KB per workgroup would keep the chain's LDS-using
    // kernels off the deep sweep's CUs (K3 136.0 / 137.1k vs 137.5 / 140.9k MLUPS, profiles/r04/ldswin)
    // f32 group slab (one cell per lane, the chain on CUs of its own): the wall split + preshift, which
    // takes the skip regions too (round 5, lbm_sweep_impl.h: SPLIT_SKIP)
    d.variant = sizeof(T) == 8       ? c->deep_variant & ~128
                : c->band_own_build ? c->deep_variant
                : slab              ? c->deep_variant & ~(128 | 8)
                                    : c->deep_variant & 1;
    if (c->band_deep_variant >= 0) d.variant = c->band_deep_variant;  // (A/B: IBLB_BAND_DEEP_VARIANT)
    d.cus = c->ncu ? (slab ? c->ncu - c->reserved_cus : c->ncu) - std::max(0, c->band_reserve) : 0;
    if (c->band_flux >= 0) {
        d.fskip0 = c->band_fy0;
        d.fskip1 = c->band_fy1;
    }
    if (c->band_par) {  // the patch outputs are the last level's (it runs beside, on the chain's stream)
        d.nskip = (int)c->band_skip.size();
        std::copy(c->band_skip.begin(), c->band_skip.end(), d.skip);
    }
    size_t ev = 0;
    hipEvent_t e0, e1;  // timing on the launch's own signals (profiling only)
    int rc = ev_kernel(c, &ev, &e0, &e1);
    if (rc) return rc;
    d.kinfo = c->deep_kinfo;
    HIP_TRY(c, launch_sweepk<T>(d, K, false, ds, e1 ? e1 : (c->band_par ? c->ev_deep : nullptr), e0));
    if (e1 && c->band_par) HIP_TRY(c, hipEventRecord(c->ev_deep, ds));
    c->deep_launches++;
    c->deep_iterations += K;
    return ev_kernel_end(c, ev, EV_SWEEPK, (long long)n * c->ny);
}

// Point indices [*lo, *hi) that may have a periodic image (m = -1 / +1) spreading into the slab's
// trapezoid columns this cycle: a slab that touches the lattice's x edge, ghost trapezoids (D > 0),
// points within the trapezoids' reach of that edge at iteration t (the cycle moves them less than a
// column per iteration; the hint only balances the merged launches' point groups, every image is
// evaluated either way, band_level_kernel)
static void wrap_range(const iblb_ctx* c, int* lo, int* hi) {
    *lo = *hi = 0;
    const int D = c->band_d, ns = c->ns;
    if (D <= 0 || ns <= 0 || (c->x_begin != 0 && c->x_begin + c->ncol != c->nx)) return;
    const float* xy = nullptr;
    if (c->sch_n > 0) xy = c->sch_x.data() + (size_t)sched_entry(c, c->t) * 2 * ns;
    else if (c->pts_host.size() >= 2 * (size_t)ns) xy = c->pts_host.data();
    if (!xy) return;
    const int margin = D + 2 * c->sweep_depth + 4;
    int a = INT_MAX, b = -1;
    for (int k = 0; k < ns; ++k) {
        const int x0 = (int)std::nearbyint((double)xy[2 * k]);
        if (x0 < margin || x0 > c->nx - 1 - margin) {
            a = std::min(a, k);
            b = k;
        }
    }
    if (b >= 0 && b + 1 - a < ns) {  // (every point: nothing to balance)
        *lo = a;
        *hi = b + 1;
    }
}

// Columns the force of level j may be spread into (the band trapezoid's [clo, chi)).  Chained
// levels: the columns level j computes; the last level stores the slab's own columns only, so a
// force left in a ghost column would never be consumed.  Merged chain: one column less at each
// ghost edge (the launch after a level clears that level's force at its own entries, one column
// narrower: the dropped column lies inside the garbage frontier, at level j columns up to
// -D+2+3j are garbage, §5 of DESIGN.md), and level K-2 only where the last level's cells and the
// nodes of its force pull: columns -3 .. ncol+2 (a point that forces column 0 has x0 >= -1, so its
// nodes start at x0-1 >= -2; their pulls reach -3, where the level's collide is recomputed, so the
// level's force is needed from column -3); the last launch clears those outside its own.
static void force_clip(const iblb_ctx* c, int j, bool merged, int* clo, int* chi) {
    const int K = c->sweep_depth, D = c->band_d, n = c->ncol;
    if (j == K - 1) {
        *clo = std::max(0, -D + 1 + j);
        *chi = std::min(n, n + D - 1 - j);
    } else if (!merged) {
        *clo = -D + 1 + j;
        *chi = n + D - 1 - j;
    } else if (j == K - 2) {
        *clo = std::max(-3, -D + 2 + j);
        *chi = std::min(n + 3, n + D - 2 - j);
    } else {
        *clo = -D + 2 + j;
        *chi = n + D - 2 - j;
    }
}

// The band chain on bs.  Chained (IBLB_BAND_MERGE=0): 2K dependent launches, the IB of each level
// over every point (image) forcing the columns the level computes, then the level's one-step
// launch over the trapezoid's entries.  Merged (default): K launches, level j's launch also
// evaluating level j+1's force (band_level_kernel: its point groups recompute level j's collide
// over their nodes' pulls), into three force buffers used in turn (level j: j % 3; the main dense
// force is buffer 0); level j's force is read, not consumed, by its launch (the point groups read it
// too) and cleared by the next launch.  The deep sweep on ds; the last level after the deep sweep
// (on ds, right behind it) and, when it stores a slab's edge columns, after the boundary sweeps
// (ev_bnd).  c->band_end is recorded on ds at the end (by the last level's own completion where it
// launches).
template <typename T>
static int band_chain(iblb_ctx* c, int K, const T* A, T* B, T* const S[2], bool slab, hipStream_t bs, hipStream_t ds,
                      const std::function<int()>& after_ib0) {
    int rc;
    const int D = c->band_d;
    const bool merged = c->band_merged && c->bf_alloc;
    double* fd[3] = {c->fdense, c->bfd[0], c->bfd[1]};
    uint8_t* fl[3] = {c->flags, c->bfl[0], c->bfl[1]};
    int clo0, chi0;
    force_clip(c, 0, merged, &clo0, &chi0);
    int wlo = 0, whi = 0;
    if (c->wrap_split) wrap_range(c, &wlo, &whi);
    if (c->ib_state == IB_PENDING) {  // force^t from g^t
        size_t ev = 0;
        if ((rc = ev_begin(c, &ev, bs))) return rc;
        // (bx_dev: its start tells the comm stream's boundary sweeps that the exchange before it landed)
        if ((rc = ib_ghost(c, A, D, clo0, chi0, pts_s(c), pts_us(c), pts_eps(c), 0, bs, c->bx_dev ? c->sig + 24 : nullptr,
                           c->bx_n, wlo, whi)))
            return rc;
        if ((rc = ev_end(c, ev, EV_IB, 0, bs))) return rc;
        c->ib_state = IB_READY;
    } else if (D > 0) {
        // force^t was evaluated before the cycle (a reader, new points, a one-step iteration) for the
        // slab's own columns only: level 0 of the ghost trapezoids needs it in the ghost columns too
        if ((rc = ib_ghost(c, A, D, clo0, 0, pts_s(c), pts_us(c), pts_eps(c), 0, bs))) return rc;
        if ((rc = ib_ghost(c, A, D, c->ncol, chi0, pts_s(c), pts_us(c), pts_eps(c), 0, bs))) return rc;
    }
    // a lone slab's deep sweep after the level-0 IB (a group slab's: band_step)
    if (!slab && (rc = band_deep<T>(c, K, ds))) return rc;
    // the launch arguments of level j (merged: its launch also evaluates level j+1's force)
    auto level = [&](int j) {
        const T* src = j == 0 ? A : S[(j - 1) & 1];
        T* dst = j == K - 1 ? B : S[j & 1];
        FusedArgs<T> a{};
        a.src = src;
        a.dst = dst;
        a.L = c->L;
        a.H = ghost_halo<T>(c, src);
        a.cols = c->band_tab;
        a.col_begin = c->band_off[j];
        a.col_step = 1;
        a.ncols = c->band_n[j];
        a.nch = c->nch;
        a.row_tab = 1;
        a.nchl = c->band_nchl[j];
        a.store_rows = j == K - 1;  // the last level writes g^{t+K}: patch output rows only
        a.vhalf = c->band_vhalf;  // the plan's chunks are 64 * V/2 rows then
        a.flags = merged ? fl[j % 3] : c->flags;
        a.fdense = merged ? fd[j % 3] : c->fdense;
        a.fplane = c->fplane;
        a.flux_col = c->band_flux;  // rows [fy0, fy1) of the flux column, every level
        a.flux_norm = c->cfg.flux_norm;
        a.Q = c->d_Q;
        a.c = c->coef;
        a.k = c->kc;
        a.variant = c->variant;
        a.probe = c->probe_level;
        if (merged) {
            if (j > 0) {  // the force of level j-1, read by the previous launch
                a.fdclr = fd[(j - 1) % 3];
                a.flclr = fl[(j - 1) % 3];
            }
            if (j < K - 1) {
                a.fkeep = 1;
                const float *ps, *pus;
                const int* pe;
                pts_of(c, c->t + j, &ps, &pus, &pe);  // force^{t+j+1}: the points of iteration t+j
                int clo, chi;
                force_clip(c, j + 1, true, &clo, &chi);
                a.nns = c->ns;
                a.nG = IbGhost{c->nx, c->x_begin, D, clo, chi, 0};
                a.n_s = ps;
                a.n_us = pus;
                a.n_eps = pe;
                a.fdnext = fd[(j + 1) % 3];
                a.flnext = fl[(j + 1) % 3];
                a.wlo = wlo;
                a.whi = whi;
            } else {  // level K-2's force in the ghost columns it may reach (no own entries there)
                int clo, chi;
                force_clip(c, K - 2, true, &clo, &chi);
                a.clr_w = std::max(0, std::min(-clo, chi - c->ncol));
                a.clr_lo = -a.clr_w;
                a.clr_hi = c->ncol;
                a.clr_waves = 2 * a.clr_w * c->nch;
            }
        }
        return a;
    };
    bool bnd_sub = false;  // the boundary sweeps submitted (bx_dev)
    for (int j = 0; j < K; ++j) {
        const T* src = j == 0 ? A : S[(j - 1) & 1];
        if (j > 0 && !merged) {  // force^{t+j} from the level below, with the points of iteration t+j-1
            const float *ps, *pus;
            const int* pe;
            pts_of(c, c->t + j - 1, &ps, &pus, &pe);
            int clo, chi;
            force_clip(c, j, false, &clo, &chi);
            size_t ev = 0;
            if ((rc = ev_begin(c, &ev, bs))) return rc;
            if ((rc = ib_ghost(c, src, D, clo, chi, ps, pus, pe, 0, bs, nullptr, 0, wlo, whi))) return rc;
            if ((rc = ev_end(c, ev, EV_IB, 0, bs))) return rc;
        }
        const FusedArgs<T> a = level(j);
        hipStream_t ls = bs;
        if (j == K - 1 && !c->band_par) {
            if (bs != ds) {  // behind the deep sweep, on its stream
                HIP_TRY(c, hipEventRecord(c->ev_bd, bs));
                HIP_TRY(c, hipStreamWaitEvent(ds, c->ev_bd, 0));
                ls = ds;
            }
            if (slab && D > 0) HIP_TRY(c, hipStreamWaitEvent(ls, c->ev_bnd, 0));
            if (a.ncols <= 0 && a.clr_waves <= 0) HIP_TRY(c, hipEventRecord(c->band_end, ls));
        } else if (j == K - 1) {  // PAR
            // a group slab's last level after the boundary sweeps too (they are done long before): the
            // next cycle's streams then wait for band_end alone, one barrier packet per queue fewer
            // (~5 us each on the critical path once the chain and the deep sweep are equally long)
            if (slab && bs != ds && (!c->bx_dev || bnd_sub)) {
                HIP_TRY(c, hipStreamWaitEvent(ls, c->ev_bnd, 0));
                c->bnd_in_end = true;
            }
            if (a.ncols <= 0 && a.clr_waves <= 0) HIP_TRY(c, hipEventRecord(c->band_end, ls));  // right after the chain
        }
        if (a.ncols <= 0 && a.nns <= 0 && a.clr_waves <= 0) continue;
        size_t ev = 0;
        if ((rc = ev_begin(c, &ev, ls))) return rc;
        HIP_TRY(c, launch_fused<T>(a, ls, j == K - 1 ? c->band_end : nullptr));
        if ((rc = ev_end(c, ev, EV_FUSED, (long long)a.ncols * a.nchl * 64 * (a.vhalf ? c->V / 2 : c->V), ls))) return rc;
        // bx_dev: the boundary sweeps after their producer (the level-0 IB) and after the first level,
        // so that their host-side submission does not delay the chain's first launches
        if (j == 0 && c->bx_dev && !bnd_sub) {
            bnd_sub = true;
            if ((rc = after_ib0())) return rc;
        }
    }
    if (c->bx_dev && !bnd_sub && (rc = after_ib0())) return rc;  // (no level-0 launch)
    return IBLB_OK;
}

// One band cycle.  A lone slab: the chain (on bs) beside the deep sweep (on ds; D > 0: the chain
// first fills the ghost columns with periodic copies), the last level on ds right behind the deep
// sweep.  Consecutive cycles stay on the two streams: the next deep sweep follows the last level
// on ds in stream order and the next chain waits for it (band_end), so a cycle costs two cross-queue
// waits (K3 timeline, profiles/r03k: joining both streams into the context's stream and starting
// the next cycle from there left 30-40 us of idle chip per cycle); band_join joins them when the
// run of cycles ends.  A slab of an RCCL group additionally:
//   bs:      after boundary(t-K) (it wrote columns the cycle reads) and the last cycle: exchange(t,
//            band_x columns) -> ev_x -> the chain (its trapezoids may read ghost columns)
//   comm:    ev_x -> boundary sweeps [0, K), [ncol-K, ncol) -> ev_bnd
//   ds:      after boundary(t-K); a non-PAR last level stores edge columns after ev_bnd
template <typename T>
static int band_step(iblb_ctx* c) {
    const int K = c->sweep_depth, D = c->band_d;
    int rc;
    const T* A = gptr<T>(c, c->cur);
    T* B = gptr<T>(c, 1 - c->cur);
    T* S[2] = {(T*)c->sbuf[0], (T*)c->sbuf[1]};
    const bool slab = !single_slab(c);
    const bool ov = c->band_st != nullptr;
    hipStream_t bs = ov ? c->band_st : c->stream, ds = ov ? c->deep_st : c->stream;
    const bool chained = ov && c->band_run;  // the previous step was a band cycle on these streams
    if (!chained) {
        if ((rc = join_comm(c))) return rc;
        if (slab) HIP_TRY(c, hipEventRecord(c->ev_pre, c->stream));
        if (ov) {
            HIP_TRY(c, hipEventRecord(c->ev_b0, c->stream));
            HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_b0, 0));
            HIP_TRY(c, hipStreamWaitEvent(ds, c->ev_b0, 0));
        }
    } else if (c->band_prev_par) {
        // the last cycle's deep sweep (ds) and last level (bs) wrote disjoint parts of g^t; each stream
        // waits for the other's: the chain reads g^t, the deep sweep reads it and overwrites the
        // buffer the last cycle's chain read.  (ev_bnd is the boundary sweeps' alone: recorded after a
        // comm-stream wait for the deep sweep as well, it saved the chain one barrier packet but put a
        // second cross-queue hop between consecutive deep sweeps, ~20 us once the chain had become
        // shorter than the deep sweep, profiles/r05/combo)
        HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_deep, 0));
        // (tried: the deep sweep's waves polling a word a signal kernel sets after the chain, instead of
        // this barrier: the signal kernel lengthened the chain by ~20 us, profiles/r05/combo4)
        HIP_TRY(c, hipStreamWaitEvent(ds, c->band_end, 0));
        if (slab && !c->bnd_in_end) {  // boundary(t-K) wrote columns both read (bnd_in_end: band_end follows it)
            HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_bnd, 0));
            HIP_TRY(c, hipStreamWaitEvent(ds, c->ev_bnd, 0));
        }
    } else {
        HIP_TRY(c, hipStreamWaitEvent(bs, c->band_end, 0));  // g^t complete: the last level of t-K on ds
        if (slab) {  // boundary(t-K) wrote columns both read
            HIP_TRY(c, hipStreamWaitEvent(bs, c->ev_bnd, 0));
            HIP_TRY(c, hipStreamWaitEvent(ds, c->ev_bnd, 0));
        }
    }
    c->bnd_in_end = false;  // (band_chain sets it for this cycle)
    hipStream_t cs = c->comm_stream;
    // a group slab's boundary sweeps [0, K), [ncol-K, ncol) on the comm stream, then ev_bnd
    auto boundary = [&]() -> int {
        Sweep2Args<T> b = sweep_args<T>(c, 0, c->ncol - K, c->ncol, 2, K);  // [0, K) and [ncol-K, ncol)
        b.vs = c->slab_vs;
        b.variant = c->deep_variant & ~128;  // beside the chain: no LDS window (above)
        if (c->band_flux >= 0) {
            b.fskip0 = c->band_fy0;
            b.fskip1 = c->band_fy1;
        }
        if (c->band_par) {  // the patch outputs of the edge columns are the last level's
            b.nskip = (int)c->band_skip.size();
            std::copy(c->band_skip.begin(), c->band_skip.end(), b.skip);
        }
        if (c->bx_dev) {  // every wave polls the word the level-0 IB sets when it starts (bounded)
            b.wait_seq = c->sig + 24;
            b.wait_val = c->bx_n;
            b.wait_lo = INT_MAX;
            b.wait_hi = INT_MAX;
            b.wait_err = c->sig_err;
            b.wait_ticks = c->wait_ticks;
            c->dev_wait_launches++;
        }
        HIP_TRY(c, launch_sweepk<T>(b, K, true, cs));
        HIP_TRY(c, hipEventRecord(c->ev_bnd, cs));
        return IBLB_OK;
    };
    c->bx_dev = false;
    if (slab) {
        // a group slab's deep sweep first (round 5: submitted behind the exchange, the boundary sweeps
        // and the level-0 IB it started late, profiles/r05/lag; a lone slab's streams may be unmasked,
        // where the chain's level-0 launches go first so that they are not queued behind the deep
        // sweep's workgroups: band_chain)
        if ((rc = band_deep<T>(c, K, ds))) return rc;
        // the exchange on the chain's stream, whose waits above put it after the whole last cycle (it
        // sends columns the last cycle wrote; the boundary sweeps after it overwrite columns that cycle
        // read): the chain's level-0 IB follows it in queue order.  On the comm stream the chain waited
        // for it across queues, and the exchange for the last cycle's end: ~15-20 us per hop on the
        // cycle's critical path (profiles/r05/df)
        if ((rc = exchange(c, bs, c->band_x))) return rc;
        // the boundary sweeps need the exchange: with the device words (PAR, reserved CUs, a level-0 IB
        // over the points) the level-0 IB's first lane signals it when the kernel starts and the boundary
        // sweeps, submitted after it, poll -- no marker packet between the exchange and the level-0 IB
        c->bx_dev = ov && c->sig && c->reserved_cus > 0 && c->edge_flag && c->band_par && c->ib_state == IB_PENDING &&
                    c->ns > 0;
        if (c->bx_dev) {
            ++c->bx_n;
        } else {
            HIP_TRY(c, hipEventRecord(c->ev_x, bs));
            HIP_TRY(c, hipStreamWaitEvent(cs, c->ev_x, 0));
            if ((rc = boundary())) return rc;
        }
    }
    if (D > 0 && !slab && (rc = fill_ghosts_periodic(c, c->cur, D, bs))) return rc;
    // the end of the cycle (ds: deep sweep and last level, after the chain), recorded by the last
    // level's completion signal: the pinned table slot may be reused once every launch of this cycle
    // has read it, and the next cycle's chain starts after it (a marker packet between the last
    // level and the next deep sweep left ~7 us of idle queue per cycle, profiles/r03ch2)
    c->band_end = c->band_pin_ev[c->band_pin_cur];  // (the waits above took the previous cycle's)
    // (bx_dev: the boundary sweeps are submitted right after the kernel they wait for)
    if ((rc = band_chain<T>(c, K, A, B, S, slab, bs, ds, boundary))) return rc;
    c->band_prev_par = c->band_par;
    c->band_cycles++;
    if (c->band_merged && c->bf_alloc) c->band_merged_cycles++;
    if (c->band_par) c->band_par_cycles++;
    c->band_run = ov;
    if (slab) {
        c->bnd_w = D > 0 ? 0 : K;  // the edge columns of g^{t+K}: the boundary sweeps' unless a trapezoid stored them
        c->deep_chain = false;
    }
    c->cur = 1 - c->cur;
    c->t += K;
    c->ghost = 0;
    c->ib_state = IB_PENDING;
    // the force now owed is that of iteration t+K-1's points
    if (c->sch_n > 0) sched_use(c, sched_entry(c, c->t - 1));
    return IBLB_OK;
}

// The context's stream after a run of band cycles (before any other step, reader or return).
int band_join(iblb_ctx* c) {
    if (!c->band_run) return IBLB_OK;
    c->band_run = false;
    // band_end follows the whole cycle: ds waited for the chain (ev_bd) before its last level;
    // a PAR cycle ends on both streams (last level on bs, deep sweep on ds)
    HIP_TRY(c, hipStreamWaitEvent(c->stream, c->band_end, 0));
    if (c->band_prev_par) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_deep, 0));
    if (rccl_multi(c)) HIP_TRY(c, hipEventRecord(c->ev_int, c->stream));  // comm_ready's "last step"
    return IBLB_OK;
}

int band_step_any(iblb_ctx* c) { return is_f64(c) ? band_step<double>(c) : band_step<float>(c); }

int band_release(iblb_ctx* c) {
    for (hipStream_t st : {c->band_st, c->deep_st})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    c->band_st = c->deep_st = nullptr;
    for (hipEvent_t e : {c->ev_b0, c->ev_bd, c->ev_deep})
        if (e) (void)hipEventDestroy(e);
    c->ev_b0 = c->ev_bd = c->ev_deep = nullptr;
    c->band_par = c->band_prev_par = false;
    c->band_skip.clear();
    c->band_end = nullptr;
    c->band_run = false;
    c->band_pin_cur = -1;
    for (int i = 0; i < BAND_PIN_SLOTS; ++i) {
        if (c->band_pin_ev[i]) (void)hipEventDestroy(c->band_pin_ev[i]);
        if (c->band_pin[i]) (void)hipHostFree(c->band_pin[i]);
        c->band_pin_ev[i] = nullptr;
        c->band_pin[i] = nullptr;
    }
    if (c->s_alloc) (void)hipFree(c->s_alloc);
    c->s_alloc = nullptr;
    if (c->bf_alloc) (void)hipFree(c->bf_alloc);
    if (c->bfl_alloc) (void)hipFree(c->bfl_alloc);
    c->bf_alloc = nullptr;
    c->bfl_alloc = nullptr;
    c->bfd[0] = c->bfd[1] = nullptr;
    c->bfl[0] = c->bfl[1] = nullptr;
    // the context may plan again after this: nothing above may be taken for allocated
    c->band_pin_cap = 0;
    c->band_pin_i = 0;
    c->band_reserve = 0;
    c->band_own_build = false;
    c->band_valid = false;
    c->band_b.clear();
    c->band_d = c->band_x = 0;
    c->band_tab = nullptr;
    return IBLB_OK;
}

}  // namespace iblbh
