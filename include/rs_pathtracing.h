/*
 * rs_pathtracing.h — C-ABI boundary of the MI355X-native path-tracing sample loop.
 *
 * This is what the reference's Rust host would bind with `extern "C"` to
 * replace its CPU renderer (INTEGRATION.md shows the binding).  Each entry
 * point names the reference interface it replaces (paths relative to the
 * dkarpushkin/rs-pathtracing checkout).  Plain pointers and sizes only; no
 * exception or abort crosses this boundary: every call returns a status
 * (PT_OK = 0, negative = error) and pt_last_error() gives the message of the
 * last failing call on the calling thread.
 *
 * Buffers: colour buffers are `Vec<Vector3d>` laid out as w*h*3 doubles,
 * row-major, index x + y*w, y = 0 at the top (src/camera/ray_caster.rs:35),
 * linear radiance (no gamma, no clamp) — the buffer render_step fills in
 * src/renderer/step_by_step.rs:115-117.
 */
#ifndef RS_PATHTRACING_H
#define RS_PATHTRACING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_ERR_INVALID -1     /* bad argument / unknown material name           */
#define PT_ERR_PARSE -2       /* JSON syntax or schema (serde_json::Error)        */
#define PT_ERR_UNSUPPORTED -3 /* valid reference JSON the GPU path does not take  */
#define PT_ERR_HIP -4         /* HIP runtime failure                               */
#define PT_ERR_STATE -5       /* call out of order (e.g. step before start)       */
#define PT_ERR_IO -6          /* unreadable / corrupt file (pt_checkpoint_load)   */

/* shape kinds */
#define PT_SPHERE 0    /* src/world/shapes/mod.rs:304-399 */
#define PT_RECTANGLE 1 /* src/world/shapes/mod.rs:150-221 */
#define PT_CUBE 2      /* src/world/shapes/mod.rs:223-302 */
#define PT_MARCH 3     /* RayMarchingShape, src/world/shapes/ray_marching.rs:10-110 */
#define PT_TORUS 4     /* src/world/shapes/mod.rs:400-494 */
#define PT_FUNC_HEART 0 /* ShapeFunctions, ray_marching.rs:121-520 */
#define PT_FUNC_SINE 1
#define PT_FUNC_STAR 2
#define PT_FUNC_DUPIN_CYCLIDE 3
#define PT_FUNC_HUNTS_SURFACE 4
#define PT_FUNC_CUSHION 5

/* material kinds (src/world/material.rs) */
#define PT_LAMBERTIAN 0
#define PT_METAL 1
#define PT_DIELECTRIC 2
#define PT_DIFFUSE_LIGHT 3
#define PT_EMPTY 4

typedef struct pt_scene pt_scene;
typedef struct pt_renderer pt_renderer;

/* Scene::from_json options.  The reference appends ~480 spheres drawn from an
 * unseeded thread_rng (src/world/json_models.rs:44, 50-133); here the draw is
 * seeded so a scene is reproducible, and it can be switched off. */
/* ImageTexture decoding: the reference calls image::open(image_filename) and
 * into_rgba8() at deserialization (src/world/texture.rs:119-130).  A loader
 * returns PT_OK with a width x height RGBA8 row-major buffer that stays valid
 * until pt_scene_create_from_json returns (the library copies it), or
 * PT_ERR_UNSUPPORTED to decline the file.  Without a loader, or for a
 * declined file, the built-in reader takes binary PPM (P6, maxval 255). */
typedef int (*pt_image_loader)(void *user, const char *filename, uint32_t *width, uint32_t *height,
                               const uint8_t **rgba8);

/* The struct is versioned by struct_size, which the library honours: it reads
 * no byte at or past opts + struct_size.  A caller sets struct_size =
 * sizeof(pt_scene_opts) of the header it was compiled against (or uses
 * PT_SCENE_OPTS_INIT).  struct_size == 0 is a caller built against 0.1.0 or
 * 0.2.0, where this field was `reserved` (always 0): 0.1.0's struct was the 16
 * bytes {random_spheres, reserved, seed}, 0.2.0's added load_image and
 * image_user, and a 0 cannot tell the two apart, so 0 reads the 16 bytes both
 * have and never a loader (ABI version 4; a 0.2.0 caller's ImageTexture files
 * then go to the built-in PPM reader).  An image loader is used only with a
 * struct_size that covers it.  A size between 1 and 15 is rejected
 * (PT_ERR_INVALID); a size of 16 to 31 reads only the fields it covers (16: no
 * loader); fields a newer caller appends past sizeof(pt_scene_opts) are
 * ignored. */
typedef struct {
    uint32_t random_spheres; /* 1 = reference behaviour (default), 0 = JSON shapes only */
    uint32_t struct_size;    /* sizeof(pt_scene_opts); 0 = a 0.1.0 / 0.2.0 caller: its first 16 bytes only */
    uint64_t seed; /* seed of the add_random_spheres stream and of the NoiseTexture Perlin tables */
    pt_image_loader load_image; /* NULL: built-in PPM reader (read only if struct_size covers it) */
    void *image_user;
} pt_scene_opts;
#define PT_SCENE_OPTS_MIN_SIZE 16    /* {random_spheres, struct_size, seed} */
#define PT_SCENE_OPTS_LEGACY_SIZE 16 /* what struct_size == 0 means: the bytes 0.1.0 and 0.2.0 structs share */
#define PT_SCENE_OPTS_INIT {1u, (uint32_t)sizeof(pt_scene_opts), 1u, NULL, NULL}

/* Camera (src/camera/mod.rs:36-46).  fov in radians, as Camera::new takes it. */
typedef struct {
    double position[3], direction[3], up[3], right[3];
    double fov, focal_length;
} pt_camera;

/* Realized shape record (introspection / parity).  Matrices are 4x4 row-major. */
typedef struct {
    int32_t type, material, inverse_normal, depth, func, pad0;
    double direct[16], inverse[16];
    double x0, y0, x1, y1, step;
    double a, b, c, d, sphere_radius; /* ray-marched function parameters (JSON) */
    double radius, tube_radius;       /* Torus */
} pt_shape_info;

typedef struct {
    int32_t type;
    int32_t texture; /* -1: SolidColor (albedo / emit hold it); else the root of a non-solid texture */
    double albedo[3];
    double fuzz, ior;
    double emit[3];
} pt_material_info;

/* RayHit (src/world/ray.rs:21-29) for the closest_hit probe. */
typedef struct {
    double t;
    double point[3];
    double normal[3];
    int32_t front_face, shape, material, pad0;
} pt_hit;

/* ---- scene: Scene::from_json (src/world/mod.rs:46-49) ------------------ */
int pt_scene_create_from_json(const char *json, size_t len, const pt_scene_opts *opts, pt_scene **out);
void pt_scene_destroy(pt_scene *scene);
/* Scene::camera (src/world/mod.rs:193-197) */
int pt_scene_camera(const pt_scene *scene, pt_camera *out);
int pt_scene_num_shapes(const pt_scene *scene);
int pt_scene_get_shape(const pt_scene *scene, int index, pt_shape_info *out);
int pt_scene_num_materials(const pt_scene *scene);
int pt_scene_get_material(const pt_scene *scene, int index, pt_material_info *out);

/* Camera::new (src/camera/mod.rs:71-88) */
int pt_camera_new(const double position[3], const double direction[3], const double up[3],
                  double focal_length, double fov_radians, pt_camera *out);

/* ---- renderer: trait Renderer (src/renderer/mod.rs:47-56) -------------- */
/* ThreadPoolRenderer::new(scene, thread_number, depth)
 * (src/renderer/step_by_step.rs:37): `device` (HIP ordinal, -1 = current)
 * replaces thread_number.  The scene must outlive the renderer. */
int pt_renderer_create(pt_scene *scene, int device, uint32_t depth, pt_renderer **out);
/* The same constructor with the parallelism knob spread over GPUs (the
 * thread_number of step_by_step.rs:37 -> ngpu): devices[0..ngpu) are HIP
 * ordinals (NULL: 0 .. ngpu-1; ngpu <= 0 with NULL devices: every visible
 * device; an ordinal may repeat, e.g. to rehearse the deal on one GPU).
 * Each device gets its own copy of the scene and its own stream.  A frame's
 * 16x16 tiles are dealt to the devices as to the ranks of pt_render_device
 * (logical tile k -> device k % ngpu, diagonal deal); each device renders
 * its tiles into a compact shard, the shards are copied to devices[0] over
 * the peer link (xGMI) and un-interleaved there.  render_start / render_step
 * / stop_rendering then drive all devices; the frame is bit-identical to a
 * one-device render (the RNG is keyed per (pixel, sample)). */
int pt_renderer_create_multi(pt_scene *scene, const int *devices, int ngpu, uint32_t depth, pt_renderer **out);
int pt_renderer_num_devices(const pt_renderer *r);
/* Peer access of a multi-device renderer.  Create enables it both ways
 * between devices[0] and every other distinct device that can reach it
 * (hipDeviceCanAccessPeer, then hipDeviceEnablePeerAccess; "already enabled"
 * counts as enabled), so the shard copies go device to device over xGMI.  A
 * pair that cannot be enabled still works: hipMemcpyPeerAsync stages it.
 * *pairs = distinct (devices[0], devices[k]) pairs, *enabled = those with
 * peer access on both ways.  A repeated ordinal is no pair. */
int pt_renderer_peer_access(const pt_renderer *r, int *pairs, int *enabled);
/* Tuning knobs of the render engines (not part of the reference; defaults are
 * the measured optimum): "engine" (0 auto, 1 megakernel,
 * 2 wavefront), "mega_waves", "diag", "wf_slots", "wf_paths", "wf_min_chunks",
 * "wf_bounce_waves", "wf_march_slice", "wf_walk", "bvh_leaf" (shapes per BVH
 * leaf: setting it rebuilds the BVH on every device).  (ABI 4's
 * "wf_march_blocks_per_cu", "wf_side_priority", "wf_pingpong", "wf_stagger"
 * and "wf_tail_paths" were measured slower and removed; setting one is
 * PT_ERR_INVALID.)  A new renderer
 * starts from the defaults; set_option changes them for every device of the
 * renderer (not while a render_start frame is in flight).  No knob changes the
 * image: every setting renders the same bits.  pt_option_name(i) lists the
 * names (NULL past the end).  get_option also reads "bvh_nodes" (read-only:
 * nodes per octant layout of the renderer's BVH; from 32768 on, the bounce
 * runs its large-tree build, whose node slab test is f32). */
int pt_renderer_set_option(pt_renderer *r, const char *name, int64_t value);
int pt_renderer_get_option(const pt_renderer *r, const char *name, int64_t *value);
const char *pt_option_name(int index);
void pt_renderer_destroy(pt_renderer *r);
/* Renderer::start_rendering (mod.rs:48-53): queues the whole frame on the
 * GPU(s), in ~8 bands of tile rows, and returns at once.  seed keys the
 * per-(pixel, sample) RNG stream.  A frame still in flight is stopped first
 * (the GUI calls stop_rendering before every start, src/bin/main.rs:268). */
int pt_render_start(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                    uint32_t samples_number, uint64_t seed);
/* Renderer::render_step (mod.rs:54): copies every finished band of rows into
 * rgb (w*h*3 doubles) and returns 1 once the frame is complete, 0 while work
 * is pending (blocking = 0, step_by_step.rs:101-121 semantics), or blocks
 * until done (blocking = 1, thread_pool_new.rs:96-126 semantics). */
int pt_render_step(pt_renderer *r, double *rgb, int blocking);
/* render_step plus the GUI's display encode (src/bin/main.rs:281-289), done on
 * the GPU right after each band: rgba (w*h*4 bytes, R G B A per pixel) gets
 * the encoded rows of every finished band; rgb (may be NULL) the linear ones.
 * Same return values as pt_render_step. */
int pt_render_step_rgba8(pt_renderer *r, double *rgb, uint8_t *rgba, int blocking);
/* Renderer::stop_rendering (mod.rs:55): the frame in flight is abandoned.  No
 * further band is queued, and the renderer's stop flag (host-mapped, read at
 * each sample chunk's start and after each compaction) turns the launches
 * already queued into no-ops; the call returns once the device streams are
 * idle, i.e. after
 * the kernels that were running when it was called (milliseconds, not the
 * seconds two whole bands take at 4K x 4096 spp).  Bands already copied by
 * render_step stay valid; the rest of the buffer is not written.  Frames
 * queued by pt_render_device / pt_render_frame_device are not affected. */
int pt_render_stop(pt_renderer *r);

/* ---- device-resident frame (benchmarks, multi-GPU) --------------------- */
/* Renders this rank's share of the frame straight into device memory on
 * `hip_stream` (a hipStream_t; 0 = the null stream, as in every HIP call and
 * in pt_unshard_device), on the renderer's first device.  Pixels are cut into
 * 16x16 tiles; logical tile k belongs to rank k % world and sits in
 * tile row k / tiles_x at column (k % tiles_x + row) % tiles_x (a diagonal
 * deal, so a rank's columns change from row to row).  world == 1: d_out is
 * the w*h*3 frame.  world > 1: d_out holds this rank's tiles in order,
 * pt_shard_tiles(...) * 256 * 3 doubles (pixels outside the frame are 0). */
int pt_render_device(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                     uint32_t samples_number, uint64_t seed, uint32_t rank, uint32_t world,
                     double *d_out, void *hip_stream);
/* The whole frame over all of the renderer's devices (pt_renderer_create_multi)
 * into d_frame (w*h*3 doubles on the first device), ordered after the work
 * queued on hip_stream (a stream of the first device; 0 = null stream), which
 * resumes once d_frame holds the frame.  Not while a render_start frame is in
 * flight (PT_ERR_STATE). */
int pt_render_frame_device(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                           uint32_t samples_number, uint64_t seed, double *d_frame, void *hip_stream);
uint32_t pt_shard_tiles(uint32_t width, uint32_t height, uint32_t rank, uint32_t world);
/* Rebuild the frame from `world` gathered shard buffers laid out back to back,
 * each padded to pt_shard_tiles(w, h, 0, world) tiles, on HIP device `device`
 * (-1 = the calling thread's current device) and its stream hip_stream.
 * (ABI version 3 added the leading `device`; see PT_ABI_VERSION.) */
int pt_unshard_device(int device, const double *d_gathered, uint32_t width, uint32_t height, uint32_t world,
                      double *d_frame, void *hip_stream);

/* ---- resumable frames (checkpoint / resume) ----------------------------- */
/* The reference renders a frame in one go and keeps nothing between runs
 * (Renderer::render, src/renderer/mod.rs:67-114; its GUI saves only the
 * encoded image, src/bin/main.rs:281-289).  A frame here can be cut into
 * sample windows instead: pt_render_device_samples renders samples
 * [s_begin, s_end) of exactly the frame pt_render_device(..., samples_number,
 * ...) renders, into the same d_out layout.  d_out holds per-pixel running
 * sums between windows: read when s_begin > 0 (the sums of samples
 * [0, s_begin)), written as sums when s_end < samples_number and as the
 * means when s_end == samples_number.  Each sample keeps its frame-wide
 * index (its RNG key, pt_sample_key) and the sums add samples in index
 * order, so windows [0, a), [a, b), ..., [z, spp) leave d_out bit-identical to
 * one pt_render_device call.  0 <= s_begin < s_end <= samples_number, else
 * PT_ERR_INVALID.  Always runs the wavefront engine. */
int pt_render_device_samples(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                             uint32_t samples_number, uint64_t seed, uint32_t rank, uint32_t world,
                             uint32_t s_begin, uint32_t s_end, double *d_out, void *hip_stream);
/* A checkpoint file: the 8 bytes "PTCKPT01", this header, `count` doubles
 * (the running sums of one rank's d_out after samples [0, samples_done)) and
 * a 64-bit FNV-1a checksum over the preceding bytes taken as little-endian
 * 64-bit words; all little-endian.  scene_key is the caller's: any value
 * that names the scene, camera and renderer options the sums belong to (the
 * Python mirror hashes the scene JSON, the camera and the depth); a resumed
 * frame must present the same key (checked by the caller). */
typedef struct pt_checkpoint {
    uint32_t width, height, samples_number, samples_done;
    uint32_t rank, world, depth, reserved; /* reserved: 0 */
    uint64_t seed;
    uint64_t scene_key;
    uint64_t count; /* doubles of sums: width*height*3 (world 1) or pt_shard_tiles(...)*768 */
} pt_checkpoint;
/* Writes header + sums[0..count) to path (atomically: a temporary file, synced
 * to disk, renamed over it, then the directory synced, so a crash or a power
 * loss leaves the old file or the new one).  The header must be consistent (samples_done <= samples_number,
 * rank < world, count as above), else PT_ERR_INVALID. */
int pt_checkpoint_save(const char *path, const pt_checkpoint *c, const double *sums);
/* Reads path's header into *c and, when sums is not NULL, its count sums
 * (capacity: doubles available at sums; fewer than count -> PT_ERR_INVALID)
 * and checks the checksum (a header-only read checks format, header and file
 * size).  A file that is missing, short, long, of another format, with an
 * inconsistent header or a checksum mismatch -> PT_ERR_IO with a message;
 * sums is zeroed on a checksum mismatch. */
int pt_checkpoint_load(const char *path, pt_checkpoint *c, double *sums, uint64_t capacity);

/* ---- probes on the GPU (reference pub fns) ----------------------------- */
/* Scene::closest_hit (src/world/mod.rs:42-44) for n rays (origin, direction:
 * 6 doubles each).  out[i].shape = -1 on a miss. */
int pt_closest_hit(pt_renderer *r, const double *rays, size_t n, double min_t, double max_t,
                   pt_hit *out);
/* ray_color (src/renderer/mod.rs:23-45) for n rays; rng_states[i] is the
 * stream state for ray i and is advanced in place. */
int pt_ray_color(pt_renderer *r, const double *rays, uint64_t *rng_states, size_t n, uint32_t depth,
                 double *out);
/* trace_pixel_samples (src/renderer/mod.rs:151-155) for an explicit list of
 * pixel indices (x + y*w); out is n*3 means. */
int pt_trace_pixel_samples(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                           uint32_t samples_number, uint64_t seed, const uint32_t *pixels, size_t n,
                           double *out);

/* Work counters of the kernel's own traversal policy over the listed pixels
 * (a diagnostic build of the same path): counters[PT_NUM_COUNTERS] receives,
 * in order, samples, bounces, sphere/rectangle/cube/marched-shape leaf tests,
 * BVH node slabs, marched-shape box slabs, literal march steps, march jump
 * attempts, march jumps, hits, Lambertian/Metal/Dielectric scatters,
 * rejection-sampling tries, attenuation multiplies, Torus tests, marches
 * dropped by the march guard.  Used for the FLOP side
 * of the roofline. */
#define PT_NUM_COUNTERS 19
int pt_count_work(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                  uint32_t samples_number, uint64_t seed, const uint32_t *pixels, size_t n,
                  uint64_t *counters);

/* The RayMarchingShape march alone (src/world/shapes/ray_marching.rs:20-74,
 * Heart) on n object-space jobs of 8 doubles {step, passes, o[3], d[3]}:
 * t_out = the march's final t, status = 1 if the passes ended (a hit before
 * the caller's [min_t, max_t] test), 2 if the march guard dropped it, else 0,
 * iters = skipping-march iterations.  Diagnostic / parity probe. */
int pt_march_jobs(pt_renderer *r, const double *jobs, size_t n, double *t_out, int32_t *status, uint32_t *iters);

/* Marches the guard dropped since the last call (read and cleared), summed over
 * the renderer's devices.  A march that has not ended after 2^24 skipping
 * iterations (each >= 1 reference step) is one the reference would not finish
 * either — e.g. a step below the rounding of t, where t + step == t and
 * ray_marching.rs:37-51 loops forever; it is taken as a miss (the ray goes on
 * to the shape's neighbours) and counted here.  Waits for the devices.
 * PT_ERR_STATE while a render_start frame is in flight. */
int pt_march_guard_drops(pt_renderer *r, uint64_t *count);

/* What pt_render_stop did on the devices since the last call (read and
 * cleared, summed over the renderer's devices): *skipped = launches of the
 * stop-gated paths (wavefront bounce, march and sample-reduce launches,
 * megakernel blocks) that found their frame stopped and did nothing;
 * *worked = launches that found it stopped and still had work (0 unless the
 * gate is broken: every launch queued behind a fired gate must be a no-op).
 * The mechanism behind stop_rendering's latency (step_by_step.rs:73-77: the
 * workers check a flag between chunks).  Waits for the devices; PT_ERR_STATE
 * while a render_start frame is in flight. */
int pt_render_stop_stats(pt_renderer *r, uint64_t *skipped, uint64_t *worked);

/* Per-kernel launch timing of the render path (bench / roofline): returns
 * the summed HIP-event durations (ms) and launch counts per kernel kind since
 * the last call — [0] bounce, [1] march, [2] list compaction, [3] sample
 * reduce, [4] megakernel, [5] per-slot unwind before the reduce (wf_unwind;
 * until round 6 the removed wavefront tail kernel), [6] BVH walk (wf_walk) — into ms[nkinds] / launches[nkinds] (either may be
 * NULL), then turns recording on (enable = 1) or off.  Events are recorded on
 * the stream each kernel is launched on.  PT_ERR_STATE while a render_start
 * frame is in flight (its band feeder records into the same timer). */
#define PT_KERNEL_KINDS 7
int pt_kernel_timing(pt_renderer *r, int enable, double *ms, uint32_t *launches, size_t nkinds);

/* Diagnostic of the wavefront kernels: returns (and clears) the counters
 * accumulated since the last call into out[min(n, 64)] — the march kernel's
 * trips and s_memtime cycles per mix of lane phases (16 + 16), lanes per
 * phase (4), then the bounce kernel's cycles per section (list load, state
 * loads, shade, unwind, trace, march pre-check, stores; each section ended by
 * a full s_waitcnt, so the waits it causes are charged to it) — and turns the
 * instrumented build on (enable = 1) or off.  PT_ERR_STATE while a
 * render_start frame is in flight; PT_ERR_UNSUPPORTED (enable = 1) unless the
 * library was built with the instrumentation (make EXTRA=-DPT_WAVE_DIAG=1). */
int pt_wave_diag(pt_renderer *r, int enable, uint64_t *out, size_t n);

/* Diagnostic: render the whole frame (depth <= 8) with a timing build of the
 * megakernel and return wave-level s_memtime cycles summed over waves per
 * phase of its per-lane loop and pass counts: out[10] = {trace, march, select,
 * shade cycles, lane passes (sum), lane march passes (sum), max lane passes,
 * then shade split into: hit finish + material fetch, scatter, unwind/restart}. */
int pt_profile_phases(pt_renderer *r, const pt_camera *camera, uint32_t width, uint32_t height,
                      uint32_t samples_number, uint64_t seed, uint64_t *out);

/* ---- display encode and image output (src/bin/main.rs:71-82, 281-289) -- */
/* sqrt -> clamp [0, 0.999] -> *256 -> u8 (NaN -> 0), alpha 255; rgba is
 * npix*4 bytes.  Host-side. */
int pt_encode_rgba8(const double *rgb, size_t npix, uint8_t *rgba);
/* The same encode on the GPU: d_rgb / d_rgba in device memory of `device`
 * (-1 = current), d_rgba 4-byte aligned, queued on hip_stream. */
int pt_encode_rgba8_device(int device, const double *d_rgb, size_t npix, uint8_t *d_rgba, void *hip_stream);
/* image::save_buffer(path, rgba, w, h, ColorType::Rgba8) of the GUI's "F"
 * key: an RGBA8 PNG (stored deflate blocks), or binary PPM (P6, alpha
 * dropped). */
int pt_write_png(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height);
int pt_write_ppm(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height);

/* ---- RNG spec shared with the parity oracle ---------------------------- */
uint64_t pt_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample);

const char *pt_last_error(void);
const char *pt_version(void);

/* ---- ABI self-description ----------------------------------------------- */
/* PT_ABI_VERSION changes whenever an entry point's signature or a struct's
 * layout or meaning changes (3: pt_scene_opts.struct_size, pt_unshard_device's
 * leading `device`, pt_abi_layout; 4: struct_size 0 reads 16 bytes, no
 * loader).  A binding compares it with the value it was
 * written for before calling anything else. */
#define PT_ABI_VERSION 4
uint32_t pt_abi_version(void);
/* Layout of a boundary struct as the library was compiled: out[0] = sizeof,
 * out[1 + k] = offsetof of the k-th field in declaration order.  Writes
 * min(n, fields + 1) values and returns fields + 1, or PT_ERR_INVALID for an
 * unknown `which`.  A binding (ctypes, Rust #[repr(C)]) checks its own
 * declarations against it. */
#define PT_ABI_SCENE_OPTS 0    /* 5 fields */
#define PT_ABI_CAMERA 1        /* 6 fields: position, direction, up, right, fov, focal_length */
#define PT_ABI_SHAPE_INFO 2    /* 20 fields, as declared */
#define PT_ABI_MATERIAL_INFO 3 /* 6 fields */
#define PT_ABI_HIT 4           /* 7 fields */
#define PT_ABI_CHECKPOINT 5    /* 11 fields, as declared */
int pt_abi_layout(int which, uint32_t *out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
