// pt_scene.hpp — host-side scene realization: Scene::from_json
// (src/world/mod.rs:46-49 -> json_models.rs:31-48), InversableTransform
// (src/algebra/transform.rs:16-23), Camera::new (src/camera/mod.rs:71-88) and
// the ray-caster constants (src/camera/ray_caster.rs:30-48).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rs_pathtracing.h"
#include "pt_types.hpp"

namespace pt {

struct HostShape {
    int32_t type = 0, material = 0, inverse_normal = 0, depth = 4, func = 0;
    double direct[4][4], inverse[4][4];
    double x0 = 0, y0 = 0, x1 = 0, y1 = 0, step = 0;
    double radius = 0, tube_radius = 0;  // Torus
    // RayMarchingShape function parameters as in the JSON (a, b, c, d,
    // sphere_radius; unused ones 0) and the derived constants the kernels use
    double fa = 0, fb = 0, fc = 0, fd = 0, fr = 0;
};

struct HostMaterial {
    int32_t type = EMPTY;
    int32_t tex = -1;  // root texture node, -1: SolidColor (albedo / emit hold the colour)
    double albedo[3] = {0, 0, 0};
    double fuzz = 0, ior = 0;
    double emit[3] = {0, 0, 0};
};

struct Scene {
    std::vector<HostShape> shapes;
    std::vector<HostMaterial> materials;
    pt_camera camera;
    int json_shapes = 0;  // shapes from the JSON file; random spheres follow
    double background[3];  // parsed but unused, as in the reference (src/world/mod.rs:199-202)
    // non-solid textures: tree nodes, one Perlin table per NoiseTexture, images
    std::vector<DTexture> textures;
    std::vector<DPerlin> perlins;
    std::vector<DImage> images;
    std::vector<uint8_t> pixels;
};

// ImageTexture decoding (image::open, src/world/texture.rs:119-130) is the
// host's: the C-ABI caller may pass a loader; binary PPM (P6) is built in.
struct ImageSource {
    pt_image_loader load = nullptr;
    void *user = nullptr;
};

// Throws SceneError on bad input (converted to a status code at the C-ABI).
struct SceneError {
    int code;
    std::string msg;
};

Scene scene_from_json(const char *json, size_t len, bool random_spheres, uint64_t seed,
                      const ImageSource &images = ImageSource());
// Perlin::new (src/algebra/noise.rs:23-42) from the k-th NoiseTexture's stream of the scene seed.
void perlin_new(uint64_t seed, uint32_t k, DPerlin *out);

void transform_new(const double t[3], const double r[3], const double s[3], double direct[4][4],
                   double inverse[4][4]);
void camera_new(const double pos[3], const double dir[3], const double up[3], double focal, double fov,
                pt_camera *out);
// Fills the caster part of FrameParams (pos/right/up/left_top/pixel_resolution).
void caster_params(const pt_camera &cam, uint32_t width, uint32_t height, FrameParams *fp);

// RNG spec: SplitMix64 finaliser, keyed per (pixel, sample).
uint64_t mix64(uint64_t z);
uint64_t sample_key(uint64_t seed, uint64_t pixel, uint64_t sample);
double uniform_incl_scale(double lo, double hi);

DShape to_device(const HostShape &s);
DMaterial to_device(const HostMaterial &m);

}  // namespace pt
