// Development tool (not product, not a test): profiles the skipping Heart
// march on the march jobs the real cornell path produces.
//   march_prof capture <scene.json> <pixels> <spp> <jobs.bin>   run the product path (host
//                                                              build) and record every march start
//   march_prof run <jobs.bin> [n]                               replay: counters, CPU time, and
//                                                              exactness against a literal march
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

struct Job {
    double step;
    int passes, pad;
    double o[3], d[3];
};
static std::vector<Job> g_jobs;
static bool g_capture = false;
static long g_hist_adv[64], g_hist_blockmax[64], g_hist_levels[64];
static int g_cur_adv = 0, g_block_max = 0, g_cur_levels = 0;
struct Prof {
    unsigned long long lin_init, advance_loops, sir_inside, evals, iters, lin_fail_zero, lin_fail_q, lin_fail_tie, lin_fail_zone;
};
static Prof g_prof;
#define PT_MPROF(f) (g_prof.f++)
#define PT_MHOOK(what) hook_##what()
static unsigned long long g_adv0, g_lv0;
static void hook_adv_begin();
static void hook_adv_end();
static void hook_lv_begin();
static void hook_lv_end();
static void hook_block_begin();
static void hook_block_end();
#define PT_MCAPTURE(step0, passes, ox, oy, oz, dx, dy, dz)                              \
    do {                                                                                 \
        if (g_capture) g_jobs.push_back(Job{step0, passes, 0, {ox, oy, oz}, {dx, dy, dz}}); \
    } while (0)

#include "../rs-pathtracing_amd/csrc/pt_accel.hpp"
#include "../rs-pathtracing_amd/csrc/pt_device.hpp"
#include "../rs-pathtracing_amd/csrc/pt_scene.hpp"

using namespace pt;

static void hook_adv_begin() { g_adv0 = g_prof.advance_loops; }
static void hook_adv_end() {
    long k = (long)(g_prof.advance_loops - g_adv0);
    g_hist_adv[k < 63 ? k : 63]++;
    if (k > g_block_max) g_block_max = (int)k;
}
static void hook_lv_begin() { g_lv0 = g_prof.evals; }
static void hook_lv_end() {
    long k = (long)(g_prof.evals - g_lv0);
    g_hist_levels[k < 63 ? k : 63]++;
}
static void hook_block_begin() { g_block_max = 0; }
static void hook_block_end() { g_hist_blockmax[g_block_max < 63 ? g_block_max : 63]++; }

static march::FParams heartF() {
    march::FParams F{};
    F.func = march::F_HEART;
    return F;
}

// The reference march, literally (ray_marching.rs:20-74), in object space.
static bool literal_march(const Job &j, double *t_out, long *steps) {
    double start, end;
    if (!march::heart_bound(j.o[0], j.o[1], j.o[2], j.d[0], j.d[1], j.d[2], &start, &end)) return false;
    double t = start, s = j.step;
    double px = j.o[0] + j.d[0] * start, py = j.o[1] + j.d[1] * start, pz = j.o[2] + j.d[2] * start;
    double r = march::heart_f(px, py, pz);
    *steps = 0;
    for (int pass = 0; pass < j.passes; pass++) {
        for (;;) {
            if (t > end || t < start) return false;
            t += s;
            px += j.d[0] * s;
            py += j.d[1] * s;
            pz += j.d[2] * s;
            (*steps)++;
            double next = march::heart_f(px, py, pz);
            if (fabs(next - 0.0) < 1e-15) {
                *t_out = t;
                return true;
            }
            if ((r < 0.0 && next > 0.0) || (r > 0.0 && next < 0.0)) {
                s = s * -0.01;
                r = next;
                break;
            }
            r = next;
        }
    }
    *t_out = t;
    return true;
}

int main(int argc, char **argv) {
    if (argc >= 6 && !strcmp(argv[1], "capture")) {
        std::ifstream f(argv[2]);
        std::stringstream ss;
        ss << f.rdbuf();
        std::string js = ss.str();
        Scene sc = scene_from_json(js.c_str(), js.size(), true, 1);
        Accel acc = build_accel(sc, sc.json_shapes);
        std::vector<DShape> shapes;
        std::vector<DMaterial> mats;
        for (auto &s : sc.shapes) shapes.push_back(to_device(s));
        for (auto &m : sc.materials) mats.push_back(to_device(m));
        dev::Scene v{};
        v.shapes = shapes.data();
        v.mats = mats.data();
        v.nodes = acc.cnodes.data();
        v.leaf = acc.leaf.data();
        v.lin = acc.lin.data();
        v.march = acc.march.data();
        v.boxes = acc.boxes.data();
        v.nnodes = acc.nodes_per_octant();
        v.nlin = (int)acc.lin.size();
        v.nmarch = (int)acc.march.size();
        const uint32_t W = 1920, H = 1080;
        FrameParams P;
        memset(&P, 0, sizeof P);
        pt_camera cam;
        memset(&cam, 0, sizeof cam);
        cam = sc.camera;
        caster_params(cam, W, H, &P);
        P.s11 = uniform_incl_scale(-1.0, 1.0);
        P.seed = 1;
        P.width = W;
        P.height = H;
        P.spp = (uint32_t)atoi(argv[4]);
        P.depth = 8;
        // <pixels>: a count (scattered sample) or a comma-separated pixel list
        std::vector<uint64_t> list;
        if (strchr(argv[3], ',')) {
            for (char *q = argv[3]; *q;) {
                list.push_back(strtoull(q, &q, 10));
                if (*q == ',') q++;
            }
        }
        long npx = list.empty() ? atol(argv[3]) : (long)list.size();
        g_capture = true;
        Ctr ctr;
        memset(&ctr, 0, sizeof ctr);
        for (long i = 0; i < npx; i++) {
            uint64_t pix = list.empty() ? (uint64_t)(i * 2654435761ull) % (W * H) : list[i];
            dev::trace_pixel<4, true>(v, P, (uint32_t)(pix % W), (uint32_t)(pix / W), &ctr);
        }
        FILE *o = fopen(argv[5], "wb");
        fwrite(g_jobs.data(), sizeof(Job), g_jobs.size(), o);
        fclose(o);
        printf("captured %zu march jobs from %ld pixels x %u spp\n", g_jobs.size(), npx, P.spp);
        printf("counters:");
        for (int k = 0; k < C_COUNT; k++) printf(" %llu", (unsigned long long)ctr.c[k]);
        printf("\n");
        return 0;
    }
    if (argc >= 3 && !strcmp(argv[1], "run")) {
        FILE *f = fopen(argv[2], "rb");
        std::vector<Job> jobs;
        Job j;
        while (fread(&j, sizeof j, 1, f) == 1) jobs.push_back(j);
        fclose(f);
        size_t n = argc > 3 ? (size_t)atol(argv[3]) : jobs.size();
        if (n > jobs.size()) n = jobs.size();
        long lit_steps = 0, bad = 0, hits = 0;
        std::vector<double> want(n);
        std::vector<int> wh(n);
        for (size_t i = 0; i < n; i++) {
            long st;
            double t = 0;
            wh[i] = literal_march(jobs[i], &t, &st);
            want[i] = t;
            lit_steps += st;
        }
        memset(&g_prof, 0, sizeof g_prof);
        march::MarchStats ms{0, 0, 0};
        auto t0 = std::chrono::steady_clock::now();
        std::vector<int> hist(64, 0);
        double hit_it = 0, miss_it = 0, hit_tries = 0, miss_tries = 0;
        long nh = 0, nm = 0;
        for (size_t i = 0; i < n; i++) {
            const Job &q = jobs[i];
            march::MarchState m;
            march::march_begin(heartF(), q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], &m);
            unsigned long long it0 = g_prof.iters;
            uint32_t tr0 = ms.tries;
            int stt;
            long guard = 0;
            while ((stt = march::march_iter<true>(m, &ms)) == march::M_RUNNING) {
                if (++guard > 2000000) {
                    printf("RUNAWAY job %zu: step %.17g passes %d o %.17g %.17g %.17g d %.17g %.17g %.17g  t %.17g s %.17g pass %d lim %lld r %.17g\n",
                           i, q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], m.t, m.s, m.pass,
                           (long long)m.lim, m.r);
                    break;
                }
            }
            unsigned long long k = g_prof.iters - it0;
            hist[k < 63 ? k : 63]++;
            bool h = stt == march::M_DONE;
            if (h) nh++, hit_it += k, hit_tries += ms.tries - tr0;
            else nm++, miss_it += k, miss_tries += ms.tries - tr0;
            if (h != (bool)wh[i] || (h && m.t != want[i])) bad++;
            hits += h;
        }
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("jobs %zu  hits %ld  mismatches %ld  literal steps/job %.1f\n", n, hits, bad, (double)lit_steps / n);
        printf("per job: iters %.2f  steps %.2f  tries %.2f  blocks %.2f  evals %.2f  lin_init %.2f  "
               "advance_loops %.2f  sir_inside %.2f   cpu %.2f us/job\n",
               (double)g_prof.iters / n, (double)ms.steps / n, (double)ms.tries / n, (double)ms.blocks / n,
               (double)g_prof.evals / n, (double)g_prof.lin_init / n, (double)g_prof.advance_loops / n,
               (double)g_prof.sir_inside / n, dt / n * 1e6);
        printf("hit jobs: iters %.2f tries %.2f   miss jobs: iters %.2f tries %.2f\n", hit_it / nh, hit_tries / nh,
               miss_it / nm, miss_tries / nm);
        printf("lin_init fails per job: zero %.2f q %.2f tie %.2f zone %.2f\n", (double)g_prof.lin_fail_zero / n,
               (double)g_prof.lin_fail_q / n, (double)g_prof.lin_fail_tie / n, (double)g_prof.lin_fail_zone / n);
        if (argc > 4) {  // results for device comparisons: t, hit, iterations per job
            FILE *o = fopen(argv[4], "wb");
            for (size_t i = 0; i < n; i++) {
                const Job &q = jobs[i];
                march::MarchState m;
                march::MarchStats st2{0, 0, 0};
                int stt = march::M_MISS;
                double k = 0;
                if (march::march_begin(heartF(), q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], &m))
                    while ((stt = march::march_iter<false>(m, &st2)) == march::M_RUNNING) k++;
                double rec[3] = {m.t, stt == march::M_DONE ? 1.0 : 0.0, k};
                fwrite(rec, sizeof rec, 1, o);
            }
            fclose(o);
        }
        auto ph = [](const char *name, long *h) {
            long tot = 0, w = 0;
            for (int i = 0; i < 64; i++) tot += h[i], w += (long)i * h[i];
            printf("%s (mean %.2f):", name, tot ? (double)w / tot : 0.0);
            for (int i = 0; i < 64; i++)
                if (h[i]) printf(" %d:%ld", i, h[i]);
            printf("\n");
        };
        ph("advance loops per call", g_hist_adv);
        ph("max advance loops over the 4 coords of a block", g_hist_blockmax);
        ph("prefix levels per call", g_hist_levels);
        printf("iterations histogram:");
        for (int i = 0; i < 64; i++)
            if (hist[i]) printf(" %d:%d", i, hist[i]);
        printf("\n");
        return bad ? 1 : 0;
    }
    fprintf(stderr, "usage: march_prof capture <scene.json> <pixels> <spp> <jobs.bin> | run <jobs.bin> [n]\n");
    return 2;
}
