// pt_scene.cpp — Scene::from_json for the GPU path.  Parses the reference's
// serde/typetag schema, realizes every shape's InversableTransform in f64 with
// the reference's operation order, appends add_random_spheres from a seeded
// stream, and rejects (PT_ERR_UNSUPPORTED) reference JSON the kernels do not
// implement yet.  Host code; compiled with -ffp-contract=off.
#include "pt_scene.hpp"

#include <cmath>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "pt_json.hpp"

namespace pt {

using ptjson::Value;

// ---------------------------------------------------------------- RNG spec
static constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;

uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    uint64_t k = mix64(seed ^ 0x6A09E667F3BCC909ull);
    k = mix64(k + (pixel + 1) * GAMMA);
    return mix64(k + (sample + 1) * 0xD1B54A32D192ED03ull);
}

namespace {

struct Stream {  // SplitMix64 (the thread_rng stand-in), rand 0.8 conversions
    uint64_t s;
    uint64_t next() {
        s += GAMMA;
        return mix64(s);
    }
    double gen() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double uniform(double lo, double scale) {
        uint64_t bits = (next() >> 12) | (1023ull << 52);
        double v;
        std::memcpy(&v, &bits, 8);
        return (v - 1.0) * scale + lo;
    }
    // Rng::gen::<u32>: the high half of the next 64-bit output (RNG spec)
    uint32_t next_u32() { return (uint32_t)(next() >> 32); }
    // gen_range(0..n) for u32 (rand 0.8.5 UniformInt::sample_single_inclusive
    // over [0, n-1]): widening multiply, rejection above the shifted zone
    uint32_t below(uint32_t n) {
        const uint32_t zone = (n << __builtin_clz(n)) - 1u;
        for (;;) {
            const uint64_t m = (uint64_t)next_u32() * n;
            if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
        }
    }
};

// ---------------------------------------------------------------- matrices
using M4 = double[4][4];

void set_identity(M4 m) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) m[i][j] = i == j ? 1.0 : 0.0;
}
// Mul<Transform> for Transform (transform.rs:553-570): sum over k in order.
void matmul(const M4 a, const M4 b, M4 out) {
    double r[4][4];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double acc = a[i][0] * b[0][j];
            acc = acc + a[i][1] * b[1][j];
            acc = acc + a[i][2] * b[2][j];
            acc = acc + a[i][3] * b[3][j];
            r[i][j] = acc;
        }
    std::memcpy(out, r, sizeof r);
}
double radians(double deg) { return deg * (M_PI / 180.0); }  // f64::to_radians

// axis 0 = roll (x), 1 = pitch (y), 2 = yaw (z): transform.rs:364-392
void axis_rotation(int axis, double deg, M4 m) {
    double r = radians(deg);
    double c = std::cos(r), s = std::sin(r);
    set_identity(m);
    int i = axis == 0 ? 1 : 0, j = axis == 2 ? 1 : 2;
    m[i][i] = c;
    m[j][j] = c;
    if (axis == 1) {  // pitch: [c 0 s; 0 1 0; -s 0 c]
        m[i][j] = s;
        m[j][i] = -s;
    } else {  // roll / yaw: [c -s; s c]
        m[i][j] = -s;
        m[j][i] = s;
    }
}
// product of three axis rotations in the given axis order, left to right
void rotation_chain(const int order[3], const double deg[3], M4 out) {
    M4 a, b, c, ab;
    axis_rotation(order[0], deg[order[0]], a);
    axis_rotation(order[1], deg[order[1]], b);
    axis_rotation(order[2], deg[order[2]], c);
    matmul(a, b, ab);
    matmul(ab, c, out);
}

}  // namespace

// InversableTransform::new (transform.rs:16-23):
//   direct  = translate(t) * rotate(r) * scale(s),   rotate = roll*pitch*yaw
//   inverse = scale(1/s) * rotate_inverse(-r) * translate(-t), rotate_inverse = yaw*pitch*roll
void transform_new(const double t[3], const double r[3], const double s[3], double direct[4][4],
                   double inverse[4][4]) {
    static const int fwd[3] = {0, 1, 2}, bwd[3] = {2, 1, 0};
    M4 T, R, S, tmp;
    set_identity(T);
    set_identity(S);
    for (int k = 0; k < 3; k++) {
        T[k][3] = t[k];
        S[k][k] = s[k];
    }
    rotation_chain(fwd, r, R);
    matmul(T, R, tmp);
    matmul(tmp, S, direct);

    double nr[3] = {-r[0], -r[1], -r[2]};
    M4 Ti, Ri, Si;
    set_identity(Ti);
    set_identity(Si);
    for (int k = 0; k < 3; k++) {
        Ti[k][3] = -t[k];
        Si[k][k] = 1.0 / s[k];
    }
    rotation_chain(bwd, nr, Ri);
    matmul(Si, Ri, tmp);
    matmul(tmp, Ti, inverse);
}

// ------------------------------------------------------------------ camera
namespace {
struct V3 {
    double x, y, z;
};
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V3 normalize(V3 a) {
    double l = std::sqrt(dot(a, a));
    return {a.x / l, a.y / l, a.z / l};
}
V3 ld(const double *p) { return {p[0], p[1], p[2]}; }
void st(double *p, V3 a) {
    p[0] = a.x;
    p[1] = a.y;
    p[2] = a.z;
}
}  // namespace

void camera_new(const double pos[3], const double dir[3], const double up[3], double focal, double fov,
                pt_camera *out) {
    V3 d = ld(dir);
    V3 right = normalize(cross(d, ld(up)));
    st(out->position, ld(pos));
    st(out->direction, normalize(d));
    st(out->up, normalize(cross(right, d)));
    st(out->right, right);
    out->fov = fov;
    out->focal_length = focal;
}

void caster_params(const pt_camera &c, uint32_t width, uint32_t height, FrameParams *fp) {
    double f = c.focal_length;
    double center[3], lt[3];
    for (int k = 0; k < 3; k++) center[k] = c.position[k] + c.direction[k] * f;
    double aspect = (double)width / (double)height;
    double vw = std::tan(c.fov / 2.0) * f * 2.0;
    double vh = vw / aspect;
    for (int k = 0; k < 3; k++) lt[k] = (center[k] - c.right[k] * (vw / 2.0)) + c.up[k] * (vh / 2.0);
    for (int k = 0; k < 3; k++) {
        fp->pos[k] = c.position[k];
        fp->right[k] = c.right[k];
        fp->up[k] = c.up[k];
        fp->left_top[k] = lt[k];
    }
    fp->pixel_resolution = vw / (double)width;
}

// UniformFloat::new_inclusive (rand 0.8.5 distributions/uniform.rs)
double uniform_incl_scale(double lo, double hi) {
    const double max_rand = 1.0 - 2.220446049250313e-16;
    double scale = (hi - lo) / max_rand;
    while (scale * max_rand + lo > hi) {
        uint64_t b;
        std::memcpy(&b, &scale, 8);
        b -= 1;
        std::memcpy(&scale, &b, 8);
    }
    return scale;
}

DShape to_device(const HostShape &s) {
    DShape d;
    std::memset(&d, 0, sizeof d);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 4; j++) {
            d.inv[i * 4 + j] = s.inverse[i][j];
            d.dir[i * 4 + j] = s.direct[i][j];
        }
    if (s.type == RECTANGLE) {
        d.p[0] = s.x0;
        d.p[1] = s.y0;
        d.p[2] = s.x1;
        d.p[3] = s.y1;
    } else if (s.type == TORUS) {
        d.p[0] = s.radius;
        d.p[1] = s.tube_radius;
    } else if (s.type == MARCH) {
        d.p[0] = s.step;
        // constants shape_func computes from the parameters (pure, so the
        // same values): Sine/Star a; DupinCyclide a, b*b, c*d, d*d
        if (s.func == 3) {
            d.fk[0] = s.fa;
            d.fk[1] = s.fb * s.fb;
            d.fk[2] = s.fc * s.fd;
            d.fk[3] = s.fd * s.fd;
        } else {
            d.fk[0] = s.fa;
        }
        d.fradius = s.fr;
    }
    d.type = s.type;
    d.material = s.material;
    d.inverse_normal = s.inverse_normal;
    d.depth = s.depth;
    d.func = s.func;
    const double(&m)[4][4] = s.inverse;
    d.axis = s.type == SPHERE && m[0][1] == 0.0 && m[0][2] == 0.0 && m[1][0] == 0.0 && m[1][2] == 0.0 &&
             m[2][0] == 0.0 && m[2][1] == 0.0 && m[0][3] != 0.0 && m[1][3] != 0.0 && m[2][3] != 0.0;
    return d;
}
DMaterial to_device(const HostMaterial &m) {
    DMaterial d;
    std::memset(&d, 0, sizeof d);
    d.type = m.type;
    d.tex = m.tex;
    for (int k = 0; k < 3; k++) {
        d.albedo[k] = m.albedo[k];
        d.emit[k] = m.emit[k];
    }
    d.fuzz = m.fuzz;
    d.ior = m.ior;
    return d;
}

// -------------------------------------------------------------- JSON schema
namespace {

[[noreturn]] void schema(const std::string &m) { throw SceneError{PT_ERR_PARSE, m}; }
[[noreturn]] void unsupported(const std::string &m) { throw SceneError{PT_ERR_UNSUPPORTED, m}; }

const Value &field(const Value &o, const char *k) {
    if (o.kind != Value::Object) schema(std::string("expected a map holding `") + k + "`");
    const Value *v = o.find(k);
    if (!v) schema(std::string("missing field `") + k + "`");
    return *v;
}
double num(const Value &v, const char *what) {
    if (v.kind != Value::Number) schema(std::string("invalid type: ") + v.kind_name() + ", expected f64 for `" + what + "`");
    return v.num;
}
std::string str(const Value &v, const char *what) {
    if (v.kind != Value::String) schema(std::string("invalid type: ") + v.kind_name() + ", expected a string for `" + what + "`");
    return v.str;
}
// Vector3d derives Deserialize: a 3-sequence or a map {x, y, z} (src/algebra/mod.rs:23-28)
void vec3(const Value &v, double out[3], const char *what) {
    if (v.kind == Value::Array) {
        if (v.arr.size() != 3) schema(std::string("invalid length ") + std::to_string(v.arr.size()) + ", expected struct Vector3d with 3 elements for `" + what + "`");
        for (int k = 0; k < 3; k++) out[k] = num(v.arr[k], what);
        return;
    }
    if (v.kind == Value::Object) {
        out[0] = num(field(v, "x"), "x");
        out[1] = num(field(v, "y"), "y");
        out[2] = num(field(v, "z"), "z");
        return;
    }
    schema(std::string("invalid type: ") + v.kind_name() + ", expected struct Vector3d for `" + what + "`");
}
// InversableTransform's custom visitor (transform.rs:120-187): exactly the
// keys translate/rotate/scale, unknown keys and duplicates are errors.
void transform(const Value &v, HostShape &s) {
    if (v.kind != Value::Object) schema("expected struct InversableTransform");
    double t[3], r[3], sc[3];
    bool ht = false, hr = false, hs = false;
    for (auto &kv : v.obj) {
        if (kv.first == "translate") {
            if (ht) schema("duplicate field `translate`");
            vec3(kv.second, t, "translate");
            ht = true;
        } else if (kv.first == "rotate") {
            if (hr) schema("duplicate field `rotate`");
            vec3(kv.second, r, "rotate");
            hr = true;
        } else if (kv.first == "scale") {
            if (hs) schema("duplicate field `scale`");
            vec3(kv.second, sc, "scale");
            hs = true;
        } else {
            schema("unknown field `" + kv.first + "`, expected one of `translate`, `rotate`, `scale`");
        }
    }
    if (!ht) schema("missing field `translate`");
    if (!hr) schema("missing field `rotate`");
    if (!hs) schema("missing field `scale`");
    transform_new(t, r, sc, s.direct, s.inverse);
}
// Binary PPM (P6, maxval 255) -> RGBA8: the built-in ImageTexture reader.
bool read_ppm(const std::string &path, uint32_t *w, uint32_t *h, std::vector<uint8_t> *rgba) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    auto token = [&](std::string *out) {
        out->clear();
        int c = std::fgetc(f);
        for (;;) {  // whitespace and # comments
            while (c != EOF && std::isspace(c)) c = std::fgetc(f);
            if (c != '#') break;
            while (c != EOF && c != '\n') c = std::fgetc(f);
        }
        while (c != EOF && !std::isspace(c)) {
            out->push_back((char)c);
            c = std::fgetc(f);
        }
        return !out->empty();
    };
    std::string m, sw, sh, sv;
    bool ok = token(&m) && m == "P6" && token(&sw) && token(&sh) && token(&sv) && sv == "255";
    long W = ok ? std::atol(sw.c_str()) : 0, H = ok ? std::atol(sh.c_str()) : 0;
    ok = ok && W > 0 && H > 0 && W < (1l << 16) && H < (1l << 16);
    std::vector<uint8_t> rgb;
    if (ok) {
        rgb.resize((size_t)W * H * 3);
        ok = std::fread(rgb.data(), 1, rgb.size(), f) == rgb.size();
    }
    std::fclose(f);
    if (!ok) return false;
    *w = (uint32_t)W;
    *h = (uint32_t)H;
    rgba->resize((size_t)W * H * 4);
    for (size_t i = 0; i < (size_t)W * H; i++) {  // into_rgba8: opaque alpha
        (*rgba)[i * 4 + 0] = rgb[i * 3 + 0];
        (*rgba)[i * 4 + 1] = rgb[i * 3 + 1];
        (*rgba)[i * 4 + 2] = rgb[i * 3 + 2];
        (*rgba)[i * 4 + 3] = 255;
    }
    return true;
}

// Texture (src/world/texture.rs), typetag "type".  Non-solid textures become
// nodes of sc.textures in pre-order (a node, then its odd subtree, then its
// even one); the k-th NoiseTexture in that order draws its Perlin tables from
// stream k of the scene seed.
struct TexCtx {
    Scene *sc;
    uint64_t seed;
    const ImageSource *img;
};
int32_t texture_node(const Value &tex, TexCtx &cx) {
    std::string t = str(field(tex, "type"), "type");
    Scene &sc = *cx.sc;
    const int32_t id = (int32_t)sc.textures.size();
    sc.textures.push_back(DTexture{});
    DTexture d{};
    d.odd = d.even = d.aux = -1;
    if (t == "SolidColor") {  // :10-20
        d.type = TEX_SOLID;
        vec3(field(tex, "color"), d.c, "color");
    } else if (t == "CheckerTexture") {  // :22-51 (the JSON `scale` key is not a field: ignored)
        d.type = TEX_CHECKER;
        vec3(field(tex, "multipliers"), d.c, "multipliers");
        d.odd = texture_node(field(tex, "odd"), cx);
        d.even = texture_node(field(tex, "even"), cx);
    } else if (t == "UVChecker") {  // :68-87, multipliers: (f64, f64)
        d.type = TEX_UVCHECKER;
        const Value &m = field(tex, "multipliers");
        if (m.kind != Value::Array || m.arr.size() != 2) schema("invalid type, expected a tuple of size 2 for `multipliers`");
        d.c[0] = num(m.arr[0], "multipliers");
        d.c[1] = num(m.arr[1], "multipliers");
        d.odd = texture_node(field(tex, "odd"), cx);
        d.even = texture_node(field(tex, "even"), cx);
    } else if (t == "NoiseTexture") {  // :53-66, noise skipped by serde -> Perlin::new()
        d.type = TEX_NOISE;
        d.c[0] = num(field(tex, "scale"), "scale");
        d.aux = (int32_t)sc.perlins.size();
        sc.perlins.push_back(DPerlin{});
        perlin_new(cx.seed, (uint32_t)d.aux, &sc.perlins.back());
    } else if (t == "ImageTexture") {  // :89-131, image::open(image_filename).into_rgba8()
        d.type = TEX_IMAGE;
        const std::string fn = str(field(tex, "image_filename"), "image_filename");
        uint32_t w = 0, h = 0;
        std::vector<uint8_t> own;
        const uint8_t *px = nullptr;
        int rc = PT_ERR_UNSUPPORTED;
        if (cx.img->load) {
            rc = cx.img->load(cx.img->user, fn.c_str(), &w, &h, &px);
            if (rc != PT_ERR_UNSUPPORTED && (rc != PT_OK || !px || !w || !h))
                throw SceneError{PT_ERR_INVALID, "Could not open texture file: " + fn};
        }
        if (rc == PT_ERR_UNSUPPORTED) {  // no loader, or it declined: the built-in reader
            if (!read_ppm(fn, &w, &h, &own))
                throw SceneError{PT_ERR_UNSUPPORTED, "Could not open texture file: " + fn +
                                                         " (without an image loader only binary PPM is read)"};
            px = own.data();
        }
        DImage im;
        im.offset = sc.pixels.size();
        im.width = w;
        im.height = h;
        sc.pixels.insert(sc.pixels.end(), px, px + (size_t)w * h * 4);
        d.aux = (int32_t)sc.images.size();
        sc.images.push_back(im);
    } else {
        schema("unknown variant `" + t + "` of Texture");
    }
    sc.textures[id] = d;
    return id;
}
// A material's albedo / emit: SolidColor inline (tex = -1), else a tree.
int32_t texture(const Value &tex, TexCtx &cx, double solid[3]) {
    if (str(field(tex, "type"), "type") == "SolidColor") {
        vec3(field(tex, "color"), solid, "color");
        return -1;
    }
    return texture_node(tex, cx);
}
HostMaterial material(const Value &m, TexCtx &cx) {
    HostMaterial h;
    std::string t = str(field(m, "type"), "type");
    if (t == "Lambertian") {  // material.rs:35-54
        h.type = LAMBERTIAN;
        h.tex = texture(field(m, "albedo"), cx, h.albedo);
    } else if (t == "Metal") {  // :56-76
        h.type = METAL;
        h.tex = texture(field(m, "albedo"), cx, h.albedo);
        h.fuzz = num(field(m, "fuzz"), "fuzz");
    } else if (t == "Dielectric") {  // :78-116
        h.type = DIELECTRIC;
        h.ior = num(field(m, "index_of_refraction"), "index_of_refraction");
    } else if (t == "DiffuseLight") {  // :118-128
        h.type = DIFFUSE_LIGHT;
        h.tex = texture(field(m, "emit"), cx, h.emit);
    } else if (t == "EmptyMaterial") {  // :130-134
        h.type = EMPTY;
    } else {
        schema("unknown variant `" + t + "` of Material");
    }
    return h;
}

}  // namespace

// Perlin::new (src/algebra/noise.rs:23-42) on the k-th NoiseTexture's stream:
// shuffle perm_x, perm_y, perm_z (SliceRandom::shuffle: for i = 255..1, swap
// i with gen_range(0..i+1)), draw the 256 unused ranfloat values, then ranvec
// = 256 x Vector3d::random(-1, 1) (algebra/mod.rs:59-66, not normalised).
void perlin_new(uint64_t seed, uint32_t k, DPerlin *out) {
    Stream rng{mix64(seed ^ 0x50455246494E4F49ull) + (uint64_t)(k + 1) * 0xD1B54A32D192ED03ull};
    for (int a = 0; a < 3; a++) {
        for (int i = 0; i < 256; i++) out->perm[a][i] = i;
        for (uint32_t i = 255; i >= 1; i--) {
            const uint32_t j = rng.below(i + 1);
            const int32_t t = out->perm[a][i];
            out->perm[a][i] = out->perm[a][j];
            out->perm[a][j] = t;
        }
    }
    for (int i = 0; i < 256; i++) (void)rng.gen();  // ranfloat
    const double s11 = uniform_incl_scale(-1.0, 1.0);
    for (int i = 0; i < 256; i++)
        for (int c = 0; c < 3; c++) out->ranvec[i][c] = rng.uniform(-1.0, s11);
}

namespace {

// add_random_spheres (src/world/json_models.rs:50-133) with a seeded stream.
void add_random_spheres(Scene &sc, uint64_t seed) {
    Stream rng{seed};
    const double s01 = uniform_incl_scale(0.0, 1.0);
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            double cx = (double)a + 0.9 * rng.gen();
            double cz = (double)b + 0.9 * rng.gen();
            double dx = cx - 4.0, dy = 0.2 - 0.2, dz = cz - 0.0;
            if (!(std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9)) continue;
            double choice = rng.gen();
            HostMaterial m;
            if (choice < 0.8) {
                double c[3];
                for (int k = 0; k < 3; k++) c[k] = rng.uniform(0.0, s01);
                m.type = LAMBERTIAN;
                for (int k = 0; k < 3; k++) m.albedo[k] = c[k] * c[k];
            } else if (choice < 0.95) {
                double c[3];
                for (int k = 0; k < 3; k++) c[k] = rng.uniform(0.0, s01);
                m.type = METAL;
                for (int k = 0; k < 3; k++) m.albedo[k] = 0.5 * (1.0 - c[k]);
                m.fuzz = 0.5 * rng.gen();
            } else {
                m.type = DIELECTRIC;
                m.ior = 1.5;
            }
            HostShape s;
            s.type = SPHERE;
            s.material = (int32_t)sc.materials.size();
            sc.materials.push_back(m);
            const double t[3] = {cx, 0.2, cz}, r[3] = {0.0, 0.0, 0.0}, k[3] = {0.2, 0.2, 0.2};
            transform_new(t, r, k, s.direct, s.inverse);
            sc.shapes.push_back(s);
        }
    }
}

}  // namespace

Scene scene_from_json(const char *json, size_t len, bool random_spheres, uint64_t seed, const ImageSource &images) {
    Value root;
    try {
        root = ptjson::parse(json, len);
    } catch (const ptjson::ParseError &e) {
        throw SceneError{PT_ERR_PARSE, e.what()};
    }
    if (root.kind != Value::Object) schema("expected struct SceneJson");
    Scene sc;

    // camera: CameraJson -> Camera (src/camera/mod.rs:13-58)
    const Value &cam = field(root, "camera");
    double pos[3], dir[3], up[3];
    vec3(field(cam, "position"), pos, "position");
    vec3(field(cam, "direction"), dir, "direction");
    vec3(field(cam, "up"), up, "up");
    double fov = num(field(cam, "fov"), "fov");
    double focal = num(field(cam, "focal_length"), "focal_length");
    camera_new(pos, dir, up, focal, radians(fov), &sc.camera);

    vec3(field(root, "background"), sc.background, "background");

    // materials: HashMap<String, Box<dyn Material>>
    const Value &mats = field(root, "materials");
    if (mats.kind != Value::Object) schema("invalid type, expected a map for `materials`");
    std::unordered_map<std::string, int32_t> index;
    TexCtx cx{&sc, seed, &images};
    for (auto &kv : mats.obj) {
        index[kv.first] = (int32_t)sc.materials.size();  // a repeated key keeps the last value
        sc.materials.push_back(material(kv.second, cx));
    }

    // shapes: Vec<Box<dyn ShapeJson>> (typetag "type"), file order
    const Value &shapes = field(root, "shapes");
    if (shapes.kind != Value::Array) schema("invalid type, expected a sequence for `shapes`");
    for (const Value &s : shapes.arr) {
        std::string t = str(field(s, "type"), "type");
        HostShape h;
        auto mat_of = [&](const Value &o) {
            std::string name = str(field(o, "material"), "material");
            auto it = index.find(name);
            // the reference indexes the HashMap and panics (shapes/mod.rs:760)
            if (it == index.end()) throw SceneError{PT_ERR_INVALID, "unknown material `" + name + "`"};
            return it->second;
        };
        if (t == "Sphere") {  // shapes/mod.rs:741-764
            str(field(s, "name"), "name");
            transform(field(s, "transform"), h);
            h.type = SPHERE;
            h.material = mat_of(s);
            if (const Value *inv = s.find("inverse_normal")) {
                if (inv->kind != Value::Bool) schema("invalid type, expected a boolean for `inverse_normal`");
                h.inverse_normal = inv->b ? 1 : 0;
            }
        } else if (t == "Rectangle") {  // :791-816
            h.x0 = num(field(s, "x0"), "x0");
            h.y0 = num(field(s, "y0"), "y0");
            h.x1 = num(field(s, "x1"), "x1");
            h.y1 = num(field(s, "y1"), "y1");
            transform(field(s, "transform"), h);
            h.type = RECTANGLE;
            h.material = mat_of(s);
        } else if (t == "Cube") {  // :818-837
            str(field(s, "name"), "name");
            transform(field(s, "transform"), h);
            h.type = CUBE;
            h.material = mat_of(s);
        } else if (t == "BruteForsableShape") {  // ray_marching.rs:532-556
            transform(field(s, "transform"), h);
            const Value &fn = field(s, "shape");
            std::string ft = str(field(fn, "type"), "type");
            // BruteForceShapeJson variants (ray_marching.rs:559-670); the
            // Heart has no fields (its bound radii are fixed, :126-131)
            if (ft == "Heart") {
                h.func = 0;
            } else if (ft == "Sine" || ft == "Star") {
                h.func = ft == "Sine" ? 1 : 2;
                h.fa = num(field(fn, "a"), "a");
                h.fr = num(field(fn, "sphere_radius"), "sphere_radius");
            } else if (ft == "DupinCyclide") {
                h.func = 3;
                h.fa = num(field(fn, "a"), "a");
                h.fb = num(field(fn, "b"), "b");
                h.fc = num(field(fn, "c"), "c");
                h.fd = num(field(fn, "d"), "d");
                h.fr = num(field(fn, "sphere_radius"), "sphere_radius");
            } else if (ft == "HuntsSurface" || ft == "Cushion") {
                h.func = ft == "HuntsSurface" ? 4 : 5;
                h.fr = num(field(fn, "sphere_radius"), "sphere_radius");
            } else {
                schema("unknown variant `" + ft + "` of BruteForceShapeJson");
            }
            h.step = num(field(s, "step"), "step");
            // the reference marches forever with step == 0 (ray_marching.rs:33-52); refuse it
            if (!(std::isfinite(h.step) && h.step != 0.0))
                throw SceneError{PT_ERR_INVALID, "BruteForsableShape step must be finite and non-zero"};
            h.depth = 4;  // default_depth (ray_marching.rs:528-530)
            if (const Value *d = s.find("depth")) {
                if (d->kind != Value::Number || !d->is_integer || d->num < 0 || d->num > 255)
                    schema("invalid value for `depth`, expected u8");
                h.depth = (int32_t)d->num;
            }
            h.type = MARCH;
            h.material = mat_of(s);
        } else if (t == "Torus") {  // shapes/mod.rs:766-789
            str(field(s, "name"), "name");
            h.radius = num(field(s, "radius"), "radius");
            h.tube_radius = num(field(s, "tube_radius"), "tube_radius");
            transform(field(s, "transform"), h);
            h.type = TORUS;
            h.material = mat_of(s);
        } else {
            schema("unknown variant `" + t + "` of ShapeJson");
        }
        sc.shapes.push_back(h);
    }
    sc.json_shapes = (int)sc.shapes.size();
    if (random_spheres) add_random_spheres(sc, seed);
    if (sc.shapes.empty())  // BvhNode::new on an empty list panics (shapes/mod.rs:702-713)
        throw SceneError{PT_ERR_INVALID, "scene has no shapes"};
    return sc;
}

}  // namespace pt
