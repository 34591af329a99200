// Development tool (not product, not a test): profiles the skipping Heart
// march on the march jobs the real cornell path produces.
//   march_prof capture <scene.json> <pixels> <spp> <jobs.bin>   run the product path (host
//                                                              build) and record every march start
//   march_prof run <jobs.bin> [n]                               replay: counters, CPU time, and
//                                                              exactness against a literal march
#include <algorithm>
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
    unsigned long long lin_init, advance_loops, sir_inside, evals, iters, lin_fail_zero, lin_fail_q, lin_fail_tie, lin_fail_zone, lit_adds;
};
static Prof g_prof;
#define PT_MPROF(f) (g_prof.f++)
#define PT_MHOOK(what) hook_##what()
static int g_it_seg[4];
#define PT_MSEG(k) (g_it_seg[k]++)
static bool g_trace = false;
#define PT_MTRACE(guess, B, good, bmax) \
    do { if (g_trace) printf("  [try guess %.4g B %lld good %lld bmax %lld]", (double)(guess), (long long)(B), (long long)(good), (long long)(bmax)); } while (0)
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

static int g_it_adv[8], g_it_nadv, g_it_levels;
static void hook_adv_begin() { g_adv0 = g_prof.advance_loops; }
static void hook_adv_end() {
    long k = (long)(g_prof.advance_loops - g_adv0);
    if (g_it_nadv < 8) g_it_adv[g_it_nadv++] = (int)k;
    g_hist_adv[k < 63 ? k : 63]++;
    if (k > g_block_max) g_block_max = (int)k;
}
static void hook_lv_begin() { g_lv0 = g_prof.evals; }
static void hook_lv_end() {
    long k = (long)(g_prof.evals - g_lv0);
    g_it_levels += (int)k;
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
        std::vector<double> job_us(n);
        for (size_t i = 0; i < n; i++) {
            const Job &q = jobs[i];
            const auto tj = std::chrono::steady_clock::now();
            march::MarchState m;
            march::march_begin(heartF(), q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], &m);
            unsigned long long it0 = g_prof.iters;
            uint32_t tr0 = ms.tries;
            int stt;
            long guard = 0;
#ifndef PROF_EXTADV
#define PROF_EXTADV 0  // 1: the block advance done by the caller after the iteration (wf_march's coop_advance)
#endif
            while ((stt = march::march_step<true, PROF_EXTADV == 0>(m, &ms)) == march::M_RUNNING) {
                if (PROF_EXTADV && m.adv) {
                    const double s = m.s, g = m.na[0];
                    m.t = march::advance(m.t, s, g);
                    m.px = march::advance(m.px, m.dx * s, g);
                    m.py = march::advance(m.py, m.dy * s, g);
                    m.pz = march::advance(m.pz, m.dz * s, g);
                    m.na[0] = m.na[1] = m.na[2] = m.na[3] = 0.0;
                    m.adv = 0;
                    m.r = march::shape_f_k<march::F_HEART>(m.F, m.px, m.py, m.pz);
                }
                if (++guard > 2000000) {
                    printf("RUNAWAY job %zu: step %.17g passes %d o %.17g %.17g %.17g d %.17g %.17g %.17g  t %.17g s %.17g pass %d lim %lld r %.17g\n",
                           i, q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], m.t, m.s, m.pass,
                           (long long)m.lim, m.r);
                    break;
                }
            }
            job_us[i] = std::chrono::duration<double>(std::chrono::steady_clock::now() - tj).count() * 1e6;
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
        {
            std::vector<double> srt = job_us;
            std::sort(srt.begin(), srt.end());
            auto q = [&](double f) { return srt[std::min(n - 1, (size_t)(f * n))]; };
            printf("job cpu us: p50 %.2f p90 %.2f p99 %.2f p99.9 %.2f p99.99 %.2f max %.2f (job %zu)\n", q(0.5), q(0.9),
                   q(0.99), q(0.999), q(0.9999), srt[n - 1],
                   (size_t)(std::max_element(job_us.begin(), job_us.end()) - job_us.begin()));
        }
        printf("hit jobs: iters %.2f tries %.2f   miss jobs: iters %.2f tries %.2f\n", hit_it / nh, hit_tries / nh,
               miss_it / nm, miss_tries / nm);
        printf("advance literal adds per job %.2f\n", (double)g_prof.lit_adds / n);
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
                    while ((stt = march::march_step<false>(m, &st2)) == march::M_RUNNING) k++;
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
    if (argc >= 3 && !strcmp(argv[1], "trace")) {  // iteration-by-iteration log of hit jobs
        FILE *f = fopen(argv[2], "rb");
        std::vector<Job> jobs;
        Job j;
        while (fread(&j, sizeof j, 1, f) == 1) jobs.push_back(j);
        fclose(f);
        int shown = 0, want = argc > 3 ? atoi(argv[3]) : 10;
        const long only = argc > 4 ? atol(argv[4]) : -1;  // one job by index
        for (size_t i = only >= 0 ? (size_t)only : 0; i < jobs.size() && shown < want; i++) {
            const Job &q = jobs[i];
            march::MarchState m;
            march::MarchStats ms{0, 0, 0, 0};
            if (!march::march_begin(heartF(), q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], &m)) continue;
            march::MarchState m0 = m;
            int stt;
            int it = 0;
            while ((stt = march::march_step<false>(m, &ms)) == march::M_RUNNING) it++;
            if (stt != march::M_DONE) continue;
            shown++;
            printf("job %zu: %d iterations, t %.17g\n", i, it + 1, m.t);
            m = m0;
            g_trace = true;
            do {
                int pass = m.pass;
                double t0 = m.t;
                uint32_t st0 = ms.steps;
                printf(" pass %d t %.10g lim %lld:", pass, t0, (long long)m.lim);
                stt = march::march_step<true>(m, &ms);
                printf(" -> t %.10g lit %u status %d\n", m.t, ms.steps - st0, stt);
            } while (stt == march::M_RUNNING);
            g_trace = false;
        }
        return 0;
    }
    if (argc >= 3 && !strcmp(argv[1], "sim")) {
        // SIMT cost model of wf_march: waves of 64 lanes refill from their
        // share of the queue; a trip costs every code region any lane runs,
        // loops at the max trip count over the lanes.
        FILE *f = fopen(argv[2], "rb");
        std::vector<Job> jobs;
        Job j;
        while (fread(&j, sizeof j, 1, f) == 1) jobs.push_back(j);
        fclose(f);
        const double C_BASE = 30, C_REFILL = 120, C_TRY = 320, C_LEVEL = 55, C_SEG = 55, C_LIT = 45;
        struct It { unsigned char tr, lit, lv, adv[4]; };
        std::vector<std::vector<It>> rec(jobs.size());
        for (size_t i = 0; i < jobs.size(); i++) {
            const Job &q = jobs[i];
            march::MarchState m;
            march::MarchStats ms{0, 0, 0, 0};
            if (!march::march_begin(heartF(), q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], &m)) continue;
            int stt;
            do {
                g_it_nadv = 0;
                g_it_levels = 0;
                for (int k = 0; k < 8; k++) g_it_adv[k] = 0;
                for (int k = 0; k < 4; k++) g_it_seg[k] = 0;
                uint32_t t0 = ms.tries, s0 = ms.steps;
                stt = march::march_step<true>(m, &ms);
                It it;
                it.tr = ms.tries != t0;
                it.lit = ms.steps != s0;
                it.lv = (unsigned char)(g_it_levels < 255 ? g_it_levels : 255);
                for (int k = 0; k < 4; k++) it.adv[k] = (unsigned char)(g_it_adv[k] + g_it_seg[k] < 255 ? g_it_adv[k] + g_it_seg[k] : 255);
                rec[i].push_back(it);
            } while (stt == march::M_RUNNING && rec[i].size() < 100000);
        }
        const int per_wave = argc > 3 ? atoi(argv[3]) : 512;
        // policy: at most K advance segments per coordinate inline; the rest
        // resumes R segments per coordinate per later iteration
        const int KIN = argc > 4 ? atoi(argv[4]) : 1000, RR = argc > 5 ? atoi(argv[5]) : 1;
        if (KIN < 1000) {
            for (auto &R : rec) {
                std::vector<It> out;
                for (auto it : R) {
                    int rem[4], mx = 0;
                    for (int k = 0; k < 4; k++) { rem[k] = it.adv[k] > KIN ? it.adv[k] - KIN : 0; if (rem[k] > mx) mx = rem[k]; it.adv[k] = it.adv[k] > KIN ? KIN : it.adv[k]; }
                    if (mx == 0) { out.push_back(it); continue; }
                    bool lit = it.lit; it.lit = 0;  // the folded literal step moves to after the advance
                    out.push_back(it);
                    while (mx > 0) {
                        It a{0, 0, 0, {0, 0, 0, 0}};
                        mx = 0;
                        for (int k = 0; k < 4; k++) { int d = rem[k] > RR ? RR : rem[k]; a.adv[k] = d; rem[k] -= d; if (rem[k] > mx) mx = rem[k]; }
                        if (mx == 0) a.lit = lit;
                        out.push_back(a);
                    }
                }
                R.swap(out);
            }
        }
        double tot = 0, useful = 0, wc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        long trips = 0;
        for (size_t w0 = 0; w0 < jobs.size(); w0 += per_wave) {
            size_t w1 = w0 + per_wave < jobs.size() ? w0 + per_wave : jobs.size();
            size_t next = w0;
            long lane_job[64], lane_pos[64];
            for (int l = 0; l < 64; l++) {
                lane_job[l] = next < w1 ? (long)next++ : -1;
                lane_pos[l] = 0;
            }
            bool refill[64];
            for (int l = 0; l < 64; l++) refill[l] = lane_job[l] >= 0;
            for (;;) {
                bool any = false, any_ref = false, any_try = false, any_lit = false;
                int mlv = 0, madv[4] = {0, 0, 0, 0};
                double lane_cost = 0;
                for (int l = 0; l < 64; l++) {
                    if (lane_job[l] < 0) continue;
                    any = true;
                    auto &R = rec[lane_job[l]];
                    if (refill[l]) { any_ref = true; lane_cost += C_REFILL; refill[l] = false; }
                    if (lane_pos[l] < (long)R.size()) {
                        const It &it = R[lane_pos[l]];
                        lane_cost += C_BASE + it.tr * C_TRY + it.lv * C_LEVEL + it.lit * C_LIT;
                        any_try |= it.tr;
                        any_lit |= it.lit;
                        if (it.lv > mlv) mlv = it.lv;
                        for (int k = 0; k < 4; k++) { lane_cost += it.adv[k] * C_SEG; if (it.adv[k] > madv[k]) madv[k] = it.adv[k]; }
                        lane_pos[l]++;
                    }
                    if (lane_pos[l] >= (long)R.size()) {
                        lane_job[l] = next < w1 ? (long)next++ : -1;
                        lane_pos[l] = 0;
                        refill[l] = lane_job[l] >= 0;
                    }
                }
                if (!any) break;
                double c = C_BASE + any_ref * C_REFILL + any_try * C_TRY + mlv * C_LEVEL + any_lit * C_LIT;
                for (int k = 0; k < 4; k++) c += madv[k] * C_SEG;
                wc[0] += C_BASE; wc[1] += any_ref * C_REFILL; wc[2] += any_try * C_TRY; wc[3] += mlv * C_LEVEL; wc[4] += any_lit * C_LIT;
                for (int k = 0; k < 4; k++) wc[5] += madv[k] * C_SEG;
                int act = 0; for (int l = 0; l < 64; l++) act += lane_job[l] >= 0; if (act < 16) wc[6] += c;
                tot += c;
                useful += lane_cost / 64.0;
                trips++;
            }
        }
        printf("jobs %zu trips %ld  wave cost %.4g  useful %.4g  lane utilisation %.1f / 64\n", jobs.size(), trips, tot,
               useful, 64.0 * useful / tot);
        printf("wave cost: base %.3g refill %.3g try %.3g levels %.3g literal %.3g advance %.3g  (trips with <16 lanes busy: %.3g)\n",
               wc[0], wc[1], wc[2], wc[3], wc[4], wc[5], wc[6]);
        // breakdown of lane work
        double w_try = 0, w_lv = 0, w_adv = 0, w_lit = 0;
        for (auto &R : rec) for (auto &it : R) { w_try += it.tr * C_TRY; w_lv += it.lv * C_LEVEL; w_lit += it.lit * C_LIT; for (int k = 0; k < 4; k++) w_adv += it.adv[k] * C_SEG; }
        printf("lane work: try %.3g levels %.3g advance %.3g literal %.3g refill %.3g\n", w_try, w_lv, w_adv, w_lit, C_REFILL * jobs.size());
        return 0;
    }
    if (argc >= 3 && !strcmp(argv[1], "tail")) {  // per-job detail of the longest marches
        FILE *f = fopen(argv[2], "rb");
        std::vector<Job> jobs;
        Job j;
        while (fread(&j, sizeof j, 1, f) == 1) jobs.push_back(j);
        fclose(f);
        const long thr = argc > 3 ? atol(argv[3]) : 40;
        std::vector<long> hist(20, 0);
        long long tot_it = 0, tail_it = 0;
        for (size_t i = 0; i < jobs.size(); i++) {
            const Job &q = jobs[i];
            march::MarchState m;
            march::MarchStats ms{0, 0, 0, 0};
            if (!march::march_begin(heartF(), q.step, q.passes, q.o[0], q.o[1], q.o[2], q.d[0], q.d[1], q.d[2], &m)) continue;
            long k = 0;
            int stt;
            unsigned long long ev0 = g_prof.evals, al0 = g_prof.advance_loops;
            int pass_it[4] = {0, 0, 0, 0};
            while ((stt = march::march_step<true>(m, &ms)) == march::M_RUNNING) {
                k++;
                if (m.pass < 4) pass_it[m.pass]++;
            }
            tot_it += k;
            int b = 0;
            while ((1l << b) <= k && b < 19) b++;
            hist[b]++;
            if (k >= thr) {
                tail_it += k;
                if (thr >= 0 && (long)i % 1 == 0)
                    printf("job %zu iters %ld status %d steps %u tries %u blocks %u evals %llu advloops %llu per-pass %d %d %d  t %.6g s0 %g start %.6g end %.6g d %.3g %.3g %.3g o %.3g %.3g %.3g\n",
                           i, k, stt, ms.steps, ms.tries, ms.blocks, g_prof.evals - ev0, g_prof.advance_loops - al0,
                           pass_it[0], pass_it[1], pass_it[2], m.t, q.step, m.start, m.end, q.d[0], q.d[1], q.d[2],
                           q.o[0], q.o[1], q.o[2]);
            }
        }
        printf("iteration log2 histogram:");
        for (int b = 0; b < 20; b++) if (hist[b]) printf(" <%ld:%ld", 1l << b, hist[b]);
        printf("\ntotal iters %lld, in jobs >= %ld: %lld\n", tot_it, thr, tail_it);
        return 0;
    }
    fprintf(stderr, "usage: march_prof capture <scene.json> <pixels> <spp> <jobs.bin> | run <jobs.bin> [n]\n");
    return 2;
}
