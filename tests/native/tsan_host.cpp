// tsan_host.cpp — ThreadSanitizer run of the product's host code that a
// caller may drive from several threads at once: Scene::from_json (the JSON
// reader and scene realization, pt_scene.cpp / pt_json.hpp), the BVH builder
// (pt_accel.cpp) and the image writer (pt_write_png / pt_write_ppm,
// pt_image.cpp, whose CRC table is built on first use).  Built by
// `make -C tests/native tsan` with g++ -fsanitize=thread (scripts/san.sh).
// 8 threads each load cornell, build its BVH and write a PNG and a PPM; every
// thread's realized scene, tree and file must equal the first's.  Test
// infrastructure only.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../rs-pathtracing_amd/csrc/pt_accel.hpp"
#include "../../rs-pathtracing_amd/csrc/pt_scene.hpp"

extern "C" void pt_set_last_error(const char *) {}

using namespace pt;

struct Result {
    size_t shapes = 0, nodes = 0;
    double check = 0;
    std::string png, ppm;
};

static std::string slurp(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: tsan_host <scene.json> <tmpdir>\n");
        return 2;
    }
    const std::string json = slurp(argv[1]), dir = argv[2];
    const int T = 8;
    std::vector<Result> res(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            Result &r = res[t];
            Scene sc = scene_from_json(json.data(), json.size(), true, 1, ImageSource{});
            Accel acc = build_accel(sc, sc.json_shapes);
            r.shapes = sc.shapes.size();
            r.nodes = acc.cnodes.size();
            for (auto &s : sc.shapes) r.check += s.direct[0][3] + s.inverse[1][1];
            std::vector<uint8_t> rgba(64 * 48 * 4);
            for (size_t i = 0; i < rgba.size(); i++) rgba[i] = (uint8_t)(i * 7 + 3);
            const std::string png = dir + "/t" + std::to_string(t) + ".png", ppm = dir + "/t" + std::to_string(t) + ".ppm";
            if (pt_write_png(png.c_str(), rgba.data(), 64, 48) != PT_OK) return;
            if (pt_write_ppm(ppm.c_str(), rgba.data(), 64, 48) != PT_OK) return;
            r.png = slurp(png);
            r.ppm = slurp(ppm);
        });
    for (auto &t : th) t.join();
    int bad = 0;
    for (int t = 1; t < T; t++)
        if (res[t].shapes != res[0].shapes || res[t].nodes != res[0].nodes || res[t].check != res[0].check ||
            res[t].png != res[0].png || res[t].ppm != res[0].ppm || res[t].png.empty())
            bad++;
    std::printf("tsan_host: %d threads, %zu shapes, %zu BVH nodes, png %zu bytes, %d mismatches\n", T, res[0].shapes,
                res[0].nodes, res[0].png.size(), bad);
    return bad ? 1 : 0;
}
