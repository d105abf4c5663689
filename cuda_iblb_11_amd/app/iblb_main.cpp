// iblb_main.cpp — drop-in for the reference driver main.cu (binary `IBLB`, reference Makefile).
//
// Same 10 positional arguments (main.cu:284-296), the same derived parameters (main.cu:298-321),
// the same iteration sequence (cilia kinematics -> LB step -> IB, main.cu:817-934, here one
// iblb_step per iteration inside libiblb) and the same output files in the same text format:
//   <data>/Raw/<c_num>/<c_fraction>//SimLog.txt        run log            (main.cu:761-790, 1007-1060)
//   <data>//Flux/<..>-flux.dat                          it*t_scale  Q*x_scale (main.cu:612, 998-1004, 1030-1034)
//   <data>/Raw/<c_num>/<c_fraction>/<it>-fluid.dat      BigData only       (main.cu:940-971)
//   <data>/Cilia/<c_num>/<c_fraction>/<it>-cilia.dat    BigData only       (main.cu:975-994)
// Deviations: the data root is $IBLB_DATA_DIR (default "Data/") instead of the
// hard-coded Windows / ShARC paths (main.cu:591-594), its directories are created, and ShARC no
// longer selects device 3 (the device is LOCAL_RANK).
//
// Multi-GPU: launched one process per GPU (e.g. `torchrun --no-python --nproc-per-node N IBLB
// ...`), ranks split the lattice into x-slabs and exchange halos over RCCL inside libiblb; the
// RCCL id travels through a rendezvous file; rank 0 gathers the fields and writes every file.
//
// Extensions (environment): IBLB_PRECISION=f32 stores populations in float; IBLB_CHECKPOINT=<prefix>
// with IBLB_CHECKPOINT_EVERY=<iterations> writes <prefix>.rank<r> checkpoints; IBLB_RESTART=<prefix>
// resumes from them (flux file appended, not truncated).
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/iblb.h"

using namespace std;

namespace {

// main.cu:22-33
const double C_S_DRIVER = 0.577;  // the driver's C_S (the LB kernels use 0.57735)
const double l_0 = 0.000006;
const double t_0 = 0.067;
const unsigned int LENGTH = 96;
const unsigned int YDIM = 192;

double seconds() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return (double)tv.tv_sec + (double)tv.tv_usec / 1e6;
}

template <typename T>
std::string to_string_3(const T a_value, const int n = 3) {  // main.cu:255-261
    std::ostringstream out;
    out << std::setprecision(n) << a_value;
    return out.str();
}

int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

std::string env_str(const char* name, const char* dflt) {
    const char* v = getenv(name);
    return v && *v ? std::string(v) : std::string(dflt);
}

void mkdirs(const std::string& path) {
    std::string cur;
    for (size_t i = 0; i < path.size(); ++i) {
        cur += path[i];
        if (path[i] == '/' && cur.size() > 1) mkdir(cur.c_str(), 0755);
    }
    if (!cur.empty() && cur.back() != '/') mkdir(cur.c_str(), 0755);
}

int die(iblb_ctx* c, int rc, const char* what) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, iblb_last_error(c) ? iblb_last_error(c) : "");
    return 1;
}

// RCCL id from rank 0 to the others through a file (written whole, then renamed into place)
bool rendezvous(int rank, char id[IBLB_UNIQUE_ID_BYTES], std::string& path) {
    path = env_str("IBLB_RDZV", "");
    if (path.empty())
        path = "/tmp/iblb_rdzv_" + env_str("TORCHELASTIC_RUN_ID", "run") + "_" + env_str("MASTER_PORT", "0");
    const time_t t_start = time(nullptr);
    if (rank == 0) {
        if (iblb_rccl_unique_id(id) != IBLB_OK) return false;
        const std::string tmp = path + ".tmp";
        FILE* f = fopen(tmp.c_str(), "wb");
        if (!f) return false;
        const bool ok = fwrite(id, 1, IBLB_UNIQUE_ID_BYTES, f) == IBLB_UNIQUE_ID_BYTES;
        fclose(f);
        return ok && rename(tmp.c_str(), path.c_str()) == 0;
    }
    for (int tries = 0; tries < 1200; ++tries) {  // up to 120 s
        struct stat st;
        if (stat(path.c_str(), &st) == 0 && st.st_mtime >= t_start - 30) {
            FILE* f = fopen(path.c_str(), "rb");
            if (f) {
                const size_t n = fread(id, 1, IBLB_UNIQUE_ID_BYTES, f);
                fclose(f);
                if (n == IBLB_UNIQUE_ID_BYTES) return true;
            }
        }
        usleep(100000);
    }
    return false;
}

}  // namespace

int main(int argc, char* argv[]) {
    //----------------------------INITIALISING---------------------------- (main.cu:265-321)
    unsigned int c_fraction = 1;
    unsigned int c_num = 6;
    double Re = 1.0;
    unsigned int XDIM = 288;
    unsigned int T = 100000;
    unsigned int T_pow = 1;
    float T_num = 1.0;
    unsigned int ITERATIONS = T;
    unsigned int P_num = 100;
    float I_pow = 1.0;
    unsigned int INTERVAL = 500;
    unsigned int c_space = 48;
    bool ShARC = 0;
    bool BigData = 0;

    const int world = env_int("WORLD_SIZE", 1), rank = env_int("RANK", 0);
    const bool lead = rank == 0;

    if (argc < 11) {
        if (lead) cout << "Too few arguments! " << argc - 1 << " entered of 10 required. " << endl;
        return 1;
    }
    stringstream arg;
    arg << argv[1] << ' ' << argv[2] << ' ' << argv[3] << ' ' << argv[4] << ' ' << argv[5] << ' ' << argv[6] << ' '
        << argv[7] << ' ' << argv[8] << ' ' << argv[9] << ' ' << argv[10];
    arg >> c_fraction >> c_num >> c_space >> Re >> T_num >> T_pow >> I_pow >> P_num >> ShARC >> BigData;

    XDIM = c_num * c_space;
    T = nearbyint(T_num * pow(10, T_pow));
    ITERATIONS = T * I_pow;
    if (P_num == 0 || ITERATIONS / P_num == 0) {  // the reference divides by zero here (main.cu:301, 938)
        if (lead) cout << "Output interval is zero: " << P_num << " data points for " << ITERATIONS << " iterations" << endl;
        return 1;
    }
    INTERVAL = ITERATIONS / P_num;

    if (XDIM < 2 * LENGTH) {
        if (lead)
            cout << "not enough cilia in simulation! Cilia spacing of " << c_space << " requires at least "
                 << 2 * LENGTH / c_space << " cilia" << endl;
        return 1;
    }

    const double dx = 1. / LENGTH;
    const double dt = 1. / (T);
    const double SPEED = 0.8 * 1000 / T;
    const double t_scale = 1000. * dt * t_0;
    const double x_scale = 1000000. * dx * l_0;
    const double s_scale = x_scale / t_scale;
    const double TAU = (SPEED * LENGTH) / (Re * C_S_DRIVER * C_S_DRIVER) + 1. / 2.;
    const double TAU2 = 1. / (12. * (TAU - (1. / 2.))) + (1. / 2.);
    const double Ma = 1. * SPEED / C_S_DRIVER;

    time_t rawtime;
    struct tm* timeinfo;
    time(&rawtime);
    timeinfo = localtime(&rawtime);
    const std::string start_stamp = asctime(timeinfo);

    if (lead) {
        cout << start_stamp << endl;
        cout << "Initialising...\n";
    }

    const int p_step = T * c_fraction / c_num;
    const unsigned int Ns = LENGTH * c_num;
    const int size = XDIM * YDIM;

    //----------------------------CONTEXT (replaces main.cu:363-754)----------------------------
    iblb_config cfg;
    iblb_config_default(&cfg);
    cfg.nx = (int)XDIM;
    cfg.ny = (int)YDIM;
    cfg.tau = TAU;
    cfg.tau2 = TAU2;
    cfg.precision = env_str("IBLB_PRECISION", "f64") == "f32" ? IBLB_PREC_F32 : IBLB_PREC_F64;
    cfg.device = env_int("LOCAL_RANK", 0);
    cfg.max_points = (int)Ns;
    if (world > 1) {
        cfg.x_begin = (int)((long long)rank * XDIM / world);
        cfg.x_count = (int)((long long)(rank + 1) * XDIM / world) - cfg.x_begin;
    }
    iblb_ctx* ctx = nullptr;
    int rc = iblb_create(&cfg, &ctx);
    if (rc) return die(nullptr, rc, "iblb_create");
    if (world > 1) {
        char id[IBLB_UNIQUE_ID_BYTES];
        std::string rdzv;
        if (!rendezvous(rank, id, rdzv)) {
            fprintf(stderr, "rank %d: RCCL rendezvous through %s failed\n", rank, rdzv.c_str());
            return 1;
        }
        if ((rc = iblb_attach_rccl(ctx, id, world, rank))) return die(ctx, rc, "iblb_attach_rccl");
        if (lead) unlink(rdzv.c_str());  // every rank has joined the communicator
    }
    // rho = RHO_0, u = 0, force = 0, f = feq (main.cu:636-754)
    if ((rc = iblb_set_state(ctx, nullptr, nullptr, nullptr, nullptr))) return die(ctx, rc, "iblb_set_state");
    iblb_cilia cil{(int)c_num, (double)c_space, (int)T, p_step};
    if ((rc = iblb_set_cilia(ctx, &cil))) return die(ctx, rc, "iblb_set_cilia");

    const std::string ckpt = env_str("IBLB_CHECKPOINT", "");
    const int ckpt_every = env_int("IBLB_CHECKPOINT_EVERY", 0);
    const std::string restart = env_str("IBLB_RESTART", "");
    const std::string rank_sfx = ".rank" + std::to_string(rank);
    unsigned int it0 = 0;
    if (!restart.empty()) {
        if ((rc = iblb_load_checkpoint(ctx, (restart + rank_sfx).c_str()))) return die(ctx, rc, "iblb_load_checkpoint");
        long long t = 0;
        iblb_get_step(ctx, &t);
        it0 = (unsigned int)t;
    }

    //----------------------------------------DEFINE DIRECTORIES---------------------------------- (main.cu:589-631)
    std::string output_data = env_str("IBLB_DATA_DIR", "Data/");
    if (output_data.back() != '/') output_data += '/';
    const std::string raw_data = output_data + "Raw/" + to_string(c_num) + "/" + to_string(c_fraction) + "/";
    const std::string cilia_data = output_data + "Cilia/" + to_string(c_num) + "/" + to_string(c_fraction) + "/";
    std::string outfile = cilia_data;
    const std::string flux = output_data + "/Flux/" + to_string(c_fraction) + "_" + to_string(c_num) + "_" +
                             to_string(c_space) + "_" + to_string_3(Re) + "_" + to_string_3(T_num) + "x" +
                             to_string_3(T_pow) + "-flux.dat";
    const std::string parameters = raw_data + "/SimLog.txt";

    ofstream fsA, fsB, fsC;
    if (lead) {
        mkdirs(raw_data);
        mkdirs(cilia_data);
        mkdirs(output_data + "/Flux/");
        if (restart.empty()) {
            fsB.open(flux.c_str(), ofstream::trunc);
            fsB.close();
        }
        //-----------------------------------OUTPUT PARAMETERS----------------------------- (main.cu:761-790)
        fsC.open(parameters.c_str(), ofstream::trunc);
        fsC.close();
        fsC.open(parameters.c_str(), ofstream::app);
        fsC << start_stamp << endl;
        fsC << "Size: " << XDIM << "x" << YDIM << endl;
        fsC << "Iterations: " << ITERATIONS << endl;
        fsC << "Reynolds Number: " << Re << endl;
        fsC << "Relaxation times: " << TAU << ", " << TAU2 << endl;
        fsC << "Spatial step: " << dx * l_0 << "m" << endl;
        fsC << "Time step: " << dt * t_0 << "s" << endl;
        fsC << "Mach number: " << Ma << endl;
        fsC << "Phase Step: " << c_fraction << "/" << c_num << endl;
        if (BigData) fsC << "\nBig Data is ON" << endl;
        else fsC << "\nBig Data is OFF" << endl;
        if (ShARC) fsC << "Running on ShARC" << endl;
        else fsC << "Running on local GPU" << endl;
        cout << "Running Simulation...\n";
    }

    std::vector<double> rho, u;
    std::vector<float> s, u_s;
    std::vector<int> epsilon;
    if (lead && BigData) {
        rho.resize(size);
        u.resize(2 * (size_t)size);
        s.resize(2 * Ns);
        u_s.resize(2 * Ns);
        epsilon.resize(Ns);
    }

    time_t start = seconds();  // time_t as in main.cu:815
    time_t p_runtime = 0;
    double Q = 0.;

    //--------------------------ITERATION LOOP----------------------------- (main.cu:817-1024)
    // iblb_step runs whole iterations; the loop stops at every iteration the reference writes
    // output after (it % INTERVAL == 0), at it == INTERVAL and at checkpoints.
    const char* ng = getenv("IBLB_NAN_GUARD");
    const bool nan_guard = !(ng && std::string(ng) == "0");
    bool nan_warned = false;
    unsigned int it = it0;
    while (it < ITERATIONS) {
        unsigned int next = (it / INTERVAL) * INTERVAL;  // next output iteration >= it
        if (next < it) next += INTERVAL;
        if (ckpt_every > 0 && !ckpt.empty()) {
            const unsigned int c = ((it / ckpt_every) + 1) * ckpt_every - 1;  // last iteration before a save
            if (c < next) next = c;
        }
        if (next >= ITERATIONS) next = ITERATIONS - 1;
        if ((rc = iblb_step(ctx, (int)(next - it + 1)))) return die(ctx, rc, "iblb_step");
        it = next;

        //----------------------------DATA OUTPUT------------------------------ (main.cu:938-1005)
        long long bad = 0;  // non-finite populations at this output iteration
        if (it % INTERVAL == 0) {
            // not in the reference (it writes NaN fields on): a diverged run is reported at the first
            // output iteration that sees it, on every rank (the count is collective); that iteration's
            // output is written as the reference writes it, then the run stops with status 3 —
            // unless IBLB_NAN_GUARD=0, which keeps the reference's behaviour (warn once, go on)
            if ((rc = iblb_count_nonfinite(ctx, &bad))) return die(ctx, rc, "iblb_count_nonfinite");
            if (bad > 0 && !nan_warned) {
                cerr << "IBLB: the run diverged: " << bad << " non-finite populations at iteration " << it
                     << (nan_guard ? " (this iteration's output written, further iterations skipped)"
                                   : " (IBLB_NAN_GUARD=0: the run goes on, as the reference's)")
                     << endl;
                nan_warned = true;
            }
            if (BigData) {
                if ((rc = iblb_gather_macro(ctx, 0, lead ? rho.data() : nullptr, lead ? u.data() : nullptr)))
                    return die(ctx, rc, "iblb_gather_macro");
                if (lead) {
                    outfile = raw_data + to_string(it) + "-fluid.dat";
                    fsA.open(outfile.c_str());
                    for (int j = 0; j < (int)(XDIM * YDIM); j++) {
                        int x = j % XDIM;
                        int y = (j - j % XDIM) / XDIM;
                        double ab = sqrt(u[0 * size + j] * u[0 * size + j] + u[1 * size + j] * u[1 * size + j]);
                        fsA << x * x_scale << "\t" << y * x_scale << "\t" << u[0 * size + j] * s_scale << "\t"
                            << u[1 * size + j] * s_scale << "\t" << ab * s_scale << "\t" << rho[j] << endl;
                        if (x == (int)XDIM - 1) fsA << endl;
                    }
                    fsA.close();
                    if ((rc = iblb_get_lagrangian(ctx, s.data(), u_s.data(), epsilon.data())))
                        return die(ctx, rc, "iblb_get_lagrangian");
                    outfile = cilia_data + to_string(it) + "-cilia.dat";
                    fsA.open(outfile.c_str());
                    for (unsigned int k = 0; k < Ns; k++) {
                        fsA << s[2 * k + 0] * x_scale << "\t" << s[2 * k + 1] * x_scale << "\t" << u_s[2 * k + 0] * s_scale
                            << "\t" << u_s[2 * k + 1] * s_scale << "\t" << epsilon[k] << "\n";
                        if (k % 96 == 95 || s[2 * k + 0] > XDIM - 1 || s[2 * k + 0] < 1) fsA << "\n";
                    }
                    fsA.close();
                }
            }
            if ((rc = iblb_get_flux(ctx, &Q))) return die(ctx, rc, "iblb_get_flux");
            if (lead) {
                fsB.open(flux.c_str(), ofstream::app);
                fsB << it * t_scale << "\t" << Q * x_scale << endl;
                fsB.close();
            }
            if (bad > 0 && nan_guard) {
                iblb_destroy(ctx);
                return 3;
            }
        }

        if (it == INTERVAL && lead) {  // main.cu:1007-1022
            time_t cycle = seconds();
            p_runtime = (cycle - start) * (ITERATIONS / INTERVAL);
            time_t p_end = rawtime + p_runtime;
            timeinfo = localtime(&p_end);
            cout << "\nCompletion time: " << asctime(timeinfo) << endl;
            fsC << "\nCompletion time: " << asctime(timeinfo) << endl;
            fsC.close();
        }

        if (ckpt_every > 0 && !ckpt.empty() && (it + 1) % ckpt_every == 0)
            if ((rc = iblb_save_checkpoint(ctx, (ckpt + rank_sfx).c_str()))) return die(ctx, rc, "iblb_save_checkpoint");
        ++it;
    }

    if ((rc = iblb_get_flux(ctx, &Q))) return die(ctx, rc, "iblb_get_flux");
    if (lead) {
        fsB.open(flux.c_str(), ofstream::app);
        fsB << it * t_scale << "\t" << Q * x_scale << endl;
        fsB.close();

        //--------------------------RUNTIME OUTPUT---------------------------------- (main.cu:1036-1060)
        double end = seconds();
        double runtime = end - start;
        int hours(0), mins(0);
        double secs(0.);
        if (runtime > 3600) hours = nearbyint(runtime / 3600 - 0.5);
        if (runtime > 60) mins = nearbyint((runtime - hours * 3600) / 60 - 0.5);
        secs = runtime - hours * 3600 - mins * 60;
        // fsC is still open (and this open fails) unless it == INTERVAL was reached, as in the reference
        fsC.open(parameters.c_str(), ofstream::app);
        fsC << "Total runtime: ";
        if (hours < 10) fsC << 0;
        fsC << hours << ":";
        if (mins < 10) fsC << 0;
        fsC << mins << ":";
        if (secs < 10) fsC << 0;
        fsC << secs << endl;
        fsC.close();
    }
    iblb_destroy(ctx);
    return 0;
}
