// pt_render — headless renderer over the C-ABI: the reference GUI's scene -> frame -> image path without the
// window.  The reference binaries take `scene [spp [w h]]` (src/bin/main_raylib.rs:22-41), render with depth 50
// (src/bin/main.rs:229-240) and save the display-encoded frame as images/rendered.png on "F"
// (src/bin/main.rs:71-83, 281-289).  This does the same in one go, on the GPU:
//
//   pt_render scene.json [spp [w h]] [-d depth] [-s seed] [-o image.png|image.ppm] [-f frame.f64]
//             [-c checkpoint -n window_spp [-x windows]]
//
// -o: the encoded image (PNG, or PPM by extension; default rendered.png, the name of the reference's "F" save).
// -f: the linear f64 frame (w*h*3, row-major), for comparisons.
// -c/-n: a resumable frame: samples in windows of window_spp; after each window but the last the
//     running sums go to the checkpoint file; a run that finds the file resumes from it (same scene, camera,
//     depth, size, spp and seed, else it refuses).  -x stops after that many windows of this run (exit status 3,
//     the checkpoint kept): an interruption, for tests.  The finished frame is bit-identical to a run without -c.
// Exit status: 0 done, 1 error (the library's message on stderr), 2 usage, 3 stopped with a checkpoint.
#include <hip/hip_runtime_api.h>

#include <sys/stat.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/rs_pathtracing.h"

namespace {

int usage() {
    std::fprintf(stderr,
                 "usage: pt_render scene.json [spp [w h]] [-d depth] [-s seed] [-o image.png|.ppm] [-f frame.f64]\n"
                 "                 [-c checkpoint -n window_spp [-x windows]]\n");
    return 2;
}

int fail(const char *what, int rc) {
    std::fprintf(stderr, "pt_render: %s: %s (status %d)\n", what, pt_last_error(), rc);
    return 1;
}

bool read_file(const char *path, std::string *out) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out->append(buf, n);
    std::fclose(f);
    return true;
}

// 64-bit FNV-1a over bytes: the checkpoint's scene key (scene text, camera, depth)
uint64_t fnv(uint64_t h, const void *p, size_t n) {
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

bool ends_with(const std::string &s, const char *suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

}  // namespace

int main(int argc, char **argv) {
    std::vector<const char *> pos;
    uint32_t depth = 50, window = 0, stop_after = 0;
    uint64_t seed = 1;
    std::string out_img = "rendered.png", out_f64, ckpt;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto val = [&](const char *name) -> const char * {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "pt_render: %s needs a value\n", name);
                std::exit(usage());
            }
            return argv[++i];
        };
        if (a == "-d") depth = (uint32_t)std::strtoul(val("-d"), nullptr, 10);
        else if (a == "-s") seed = std::strtoull(val("-s"), nullptr, 10);
        else if (a == "-o") out_img = val("-o");
        else if (a == "-f") out_f64 = val("-f");
        else if (a == "-c") ckpt = val("-c");
        else if (a == "-n") window = (uint32_t)std::strtoul(val("-n"), nullptr, 10);
        else if (a == "-x") stop_after = (uint32_t)std::strtoul(val("-x"), nullptr, 10);
        else if (a.size() > 1 && a[0] == '-') return usage();
        else pos.push_back(argv[i]);
    }
    if (pos.empty() || pos.size() == 3 || pos.size() > 4 || (!ckpt.empty() && window == 0)) return usage();
    const uint32_t spp = pos.size() >= 2 ? (uint32_t)std::strtoul(pos[1], nullptr, 10) : 100;  // the GUI's 100
    const uint32_t w = pos.size() == 4 ? (uint32_t)std::strtoul(pos[2], nullptr, 10) : 1600;    // main.rs:26
    const uint32_t h = pos.size() == 4 ? (uint32_t)std::strtoul(pos[3], nullptr, 10) : 900;
    std::string json;
    if (!read_file(pos[0], &json)) {
        std::fprintf(stderr, "pt_render: cannot read %s\n", pos[0]);
        return 1;
    }
    pt_scene_opts opts = PT_SCENE_OPTS_INIT;
    pt_scene *scene = nullptr;
    pt_renderer *r = nullptr;
    pt_camera cam;
    int rc;
    if ((rc = pt_scene_create_from_json(json.data(), json.size(), &opts, &scene))) return fail(pos[0], rc);
    if ((rc = pt_scene_camera(scene, &cam))) return fail("camera", rc);
    if ((rc = pt_renderer_create(scene, -1, depth, &r))) return fail("renderer", rc);
    const size_t npix = (size_t)w * h;
    std::vector<double> rgb(npix * 3);
    if (ckpt.empty()) {
        if ((rc = pt_render_start(r, &cam, w, h, spp, seed)) || (rc = pt_render_step(r, rgb.data(), 1)) != 1)
            return fail("render", rc);
    } else {
        // a resumable frame: sample windows into a device buffer, the running sums checkpointed between them
        const uint64_t key = fnv(fnv(fnv(0xcbf29ce484222325ull, json.data(), json.size()), &cam, sizeof cam),
                                 &depth, sizeof depth);
        double *d_out = nullptr;
        if (hipMalloc((void **)&d_out, npix * 3 * sizeof(double)) != hipSuccess) {
            std::fprintf(stderr, "pt_render: hipMalloc failed\n");
            return 1;
        }
        uint32_t done = 0;
        pt_checkpoint c;
        // start fresh only when there is no checkpoint file; an existing one that does not load (corrupt, not a
        // checkpoint, unreadable) is an error, never overwritten
        struct stat sb;
        const bool exists = ::stat(ckpt.c_str(), &sb) == 0 || errno != ENOENT;
        if (exists && (rc = pt_checkpoint_load(ckpt.c_str(), &c, nullptr, 0)) != PT_OK) return fail(ckpt.c_str(), rc);
        if (exists) {
            if (c.width != w || c.height != h || c.samples_number != spp || c.seed != seed || c.depth != depth ||
                c.scene_key != key || c.world != 1) {
                std::fprintf(stderr, "pt_render: %s belongs to another frame\n", ckpt.c_str());
                return 1;
            }
            if ((rc = pt_checkpoint_load(ckpt.c_str(), &c, rgb.data(), rgb.size()))) return fail(ckpt.c_str(), rc);
            if (hipMemcpy(d_out, rgb.data(), rgb.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
                return 1;
            done = c.samples_done;
            std::fprintf(stderr, "pt_render: resuming at sample %u of %u\n", done, spp);
        }
        uint32_t windows = 0;
        while (done < spp) {
            const uint32_t end = spp - done > window ? done + window : spp;
            if ((rc = pt_render_device_samples(r, &cam, w, h, spp, seed, 0, 1, done, end, d_out, nullptr)))
                return fail("render window", rc);
            if (hipDeviceSynchronize() != hipSuccess) return 1;
            done = end;
            if (done == spp) break;
            if (hipMemcpy(rgb.data(), d_out, rgb.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
            std::memset(&c, 0, sizeof c);
            c.width = w;
            c.height = h;
            c.samples_number = spp;
            c.samples_done = done;
            c.rank = 0;
            c.world = 1;
            c.depth = depth;
            c.seed = seed;
            c.scene_key = key;
            c.count = rgb.size();
            if ((rc = pt_checkpoint_save(ckpt.c_str(), &c, rgb.data()))) return fail(ckpt.c_str(), rc);
            if (stop_after && ++windows >= stop_after) {
                std::fprintf(stderr, "pt_render: stopped at sample %u of %u, checkpoint %s\n", done, spp, ckpt.c_str());
                return 3;
            }
        }
        if (hipMemcpy(rgb.data(), d_out, rgb.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        (void)hipFree(d_out);
        std::remove(ckpt.c_str());
    }
    if (!out_f64.empty()) {
        FILE *f = std::fopen(out_f64.c_str(), "wb");
        if (!f || std::fwrite(rgb.data(), sizeof(double), rgb.size(), f) != rgb.size() || std::fclose(f) != 0) {
            std::fprintf(stderr, "pt_render: cannot write %s\n", out_f64.c_str());
            return 1;
        }
    }
    if (!out_img.empty()) {
        std::vector<uint8_t> rgba(npix * 4);
        if ((rc = pt_encode_rgba8(rgb.data(), npix, rgba.data()))) return fail("encode", rc);
        rc = ends_with(out_img, ".ppm") ? pt_write_ppm(out_img.c_str(), rgba.data(), w, h)
                                        : pt_write_png(out_img.c_str(), rgba.data(), w, h);
        if (rc) return fail(out_img.c_str(), rc);
    }
    std::printf("rendered %ux%u at %u spp, depth %u\n", w, h, spp, depth);
    pt_renderer_destroy(r);
    pt_scene_destroy(scene);
    return 0;
}
