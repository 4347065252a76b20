/*
 * rt.h — C ABI of the MI355X path-tracing kernel library (librt_amd.so).
 *
 * Drop-in boundary for the reference's hot path
 *     raytrace :: ToRandom m => CameraSettings -> Geometry m Material -> StdGen -> A.Matrix D Color
 *     (UnaryPlus/raytrace src/Graphics/Ray.hs:121-238)
 * The reference has no FFI of its own (pure Haskell, no `foreign import`); the entry points
 * below are what its Haskell side binds with `foreign import ccall safe` (INTEGRATION.md shows
 * the binding).  Plain C types only: no HIP or torch types cross this boundary; device
 * pointers and streams are passed as `void*` / `float*` owned by the caller.
 *
 * Scene contract.  The reference's Geometry / Material / Texture / background are closures
 * (Geometry.hs:42, Material.hs:17, Texture.hs:15, Ray.hs:57).  The caller reifies them through
 * a deep embedding of the same smart constructors and passes the FLATTENED scene:
 *   - every leaf surface (sphere / parallelogram / triangle) with rigid `transform`s baked in,
 *     its material (outermost `<$` wins), its `moving` motion and its depth-first `order`
 *     (the reference's closest-hit tie-break: earlier leaf wins on equal t, Geometry.hs:340-361);
 *   - every `constantMedium` lifted to the top level with its boundary leaves in their own set.
 * The library builds its own bounding-volume hierarchy over that list; the closest hit (and
 * therefore the image) does not depend on the tree the caller wrote.
 *
 * Precision.  By default the kernel computes in IEEE binary64, as the reference does (every
 * `Vec3` is `V3 Double`, Core.hs:29-31), and writes double output.  rt_exec.flags RT_EXEC_F32
 * selects the FP32 fast path (float output): the same algorithm, scheduling and random stream.
 *
 * Output.  Linear RGB, row-major [row][column][rgb] — row 0 is the TOP of the image — each
 * pixel the MEAN over `samples_per_pixel` samples (Ray.hs:226-232); double (default) or float
 * (RT_EXEC_F32) per channel.  Randomness is a counter-based Philox4x32-10 stream keyed by
 * `seed` and indexed by (pixel, sample, segment, event), so results are deterministic for a
 * given (scene, camera, seed, precision) and independent of the shard layout, of the device
 * list and of the GPU count.
 */
#ifndef RT_AMD_H
#define RT_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6

/* status codes */
#define RT_OK 0
#define RT_E_GENERIC (-1)
#define RT_E_INVALID (-2)      /* malformed scene/camera (reference: `error` / NaN)              */
#define RT_E_UNSUPPORTED (-3)  /* closure the device cannot evaluate; caller falls back to CPU   */
#define RT_E_HIP (-4)          /* HIP runtime failure (no device, launch failure, OOM)            */
#define RT_E_STACK (-5)        /* BVH traversal stack overflow (scene too deep)                   */

/* primitive kinds (Geometry.hs:58-176) */
#define RT_PRIM_SPHERE 0
#define RT_PRIM_PARALLELOGRAM 1
#define RT_PRIM_TRIANGLE 2

/* material kinds (Material.hs:41-129) */
#define RT_MAT_LIGHT_SOURCE 0
#define RT_MAT_PITCH_BLACK 1
#define RT_MAT_LAMBERTIAN 2
#define RT_MAT_LOMMEL_SEELIGER 3
#define RT_MAT_MIRROR 4
#define RT_MAT_METAL 5        /* param = fuzz */
#define RT_MAT_DIELECTRIC 6   /* param = index of refraction */
#define RT_MAT_TRANSPARENT 7
#define RT_MAT_ISOTROPIC 8
#define RT_MAT_ANISOTROPIC 9  /* param = Henyey-Greenstein g */

/* texture kinds (Texture.hs:18-78) */
#define RT_TEX_CONSTANT 0     /* c0 */
#define RT_TEX_CHECKER 1      /* nu, nv, c0, c1 */
#define RT_TEX_IMAGE 2        /* nu = width, nv = height, image = first texel in rt_scene.texels
                                 (row-major, row 0 = top of the image, 3 floats per texel) */
#define RT_TEX_NOISE 3        /* nu = layers; params[0] = frequency, params[1..3] = shift; c0, c1
                                 (fractal Perlin noise, needs rt_scene.perlin) */
#define RT_TEX_MARBLE 4       /* params[0..2] = stripe direction, params[3] = frequency,
                                 params[4..6] = shift (turbulence, needs rt_scene.perlin) */

/* background kinds (cs_background restricted to reifiable closures) */
#define RT_BG_CONST 0         /* c0 */
#define RT_BG_LERP_Y 1        /* (1 - a) c0 + a c1, a = 0.5 (dir.y + 1)  (`sky`, `grayFade`) */

/* rt_prim.set of the object-space leaves of instanced object b (rt_instance.blas == b) */
#define RT_SET_BLAS(b) (-1 - (b))

/* One leaf surface.  Ray.hs/Geometry.hs semantics; coordinates in world space, or in the
 * object space of an instanced object (set RT_SET_BLAS(b)). */
typedef struct rt_prim {
  int32_t kind;      /* RT_PRIM_* */
  int32_t material;  /* index into rt_scene.materials (ignored for medium boundaries; -1 allowed
                        for an instanced object's leaves when every instance of it has one)   */
  int32_t set;       /* 0 = visible surface; k >= 1 = boundary of rt_scene.media[k-1];
                        RT_SET_BLAS(b) = a leaf of instanced object b (object space)          */
  int32_t motion;    /* -1 or index into rt_scene.motions (`moving`, Geometry.hs:449-456)      */
  int32_t gid;       /* geometric identity: the same source leaf under the same transform has
                        the same gid in every set (used to skip self-intersection)          */
  int32_t order;     /* depth-first position of the leaf in the caller's tree (tie-break);
                        for an instanced object's leaf: its position inside the object        */
  int32_t uvframe;   /* -1 or index into rt_scene.uvframes: rotation R^T for sphereUV         */
  int32_t pad;
  double p[9];       /* sphere: center[3], radius, -; plane: q[3], u[3], v[3]                 */
  double uv[6];      /* plane shapes: uv0, uv1, uv2 (parallelogram: (0,0),(1,0),(0,1))         */
} rt_prim;

typedef struct rt_medium {   /* constantMedium (Geometry.hs:298-330) */
  double density;
  int32_t material;
  int32_t order;
} rt_medium;

typedef struct rt_material {
  int32_t kind;      /* RT_MAT_* */
  int32_t texture;   /* index into rt_scene.textures */
  double param;
} rt_material;

typedef struct rt_texture {
  int32_t kind;      /* RT_TEX_* */
  int32_t nu, nv;    /* checker dimensions | image width, height | noise layers */
  int32_t image;     /* image: index of its first texel in rt_scene.texels, else -1 */
  double c0[3], c1[3];
  double params[8];  /* noise / marble parameters (see RT_TEX_*) */
} rt_texture;

/* The Perlin tables of Noise.hs:21-92: the three fixed permutations (permX/Y/Z) and the 256
   gradients (`replicateM 256 randomUnitVector` evaluated with mkStdGen 666). */
typedef struct rt_perlin {
  int32_t perm[3][256];
  double grad[256][3];
} rt_perlin;

typedef struct rt_motion {
  double v0[3], v1[3];   /* world-space shift (1 - time) v0 + time v1 */
} rt_motion;

typedef struct rt_uvframe {
  double r[9];           /* row-major 3x3: object-space normal = r * world-space normal */
} rt_uvframe;

/* Two-level instancing of `transform` (Geometry.hs:382-391): one placement of an instanced
 * object (the leaves with set RT_SET_BLAS(blas), traced in object space under its own BVH).
 * The world ray enters the object through the inverse of the rigid transform m; t is unchanged
 * (rigid), hit points / normals go back through m.  The instance's leaves take depth-first
 * orders order .. order + (leaves of the object) - 1 in the tie-break. */
typedef struct rt_instance {
  int32_t blas;      /* instanced object */
  int32_t material;  /* material of every surface of this placement (the outermost `<$`), or -1:
                        the leaves' own materials */
  int32_t order;     /* depth-first order of the object's first leaf in the caller's tree */
  int32_t pad;
  double m[12];      /* object -> world, row-major 3 x 4, rigid (R^T R = I) */
} rt_instance;

typedef struct rt_scene {
  int32_t n_prims;      const rt_prim* prims;
  int32_t n_media;      const rt_medium* media;
  int32_t n_materials;  const rt_material* materials;
  int32_t n_textures;   const rt_texture* textures;
  int32_t n_motions;    const rt_motion* motions;
  int32_t n_uvframes;   const rt_uvframe* uvframes;
  int32_t n_texels;     const float* texels;      /* image textures' linear RGB, 3 floats each */
  const rt_perlin* perlin;                        /* required by noise / marble textures   */
  int32_t n_instances;  const rt_instance* instances;  /* two-level instancing (may be 0)  */
} rt_scene;

typedef struct rt_redirect_target {   /* cs_redirectTargets element (p, q, u, v) */
  double prob;
  double q[3], u[3], v[3];
} rt_redirect_target;

/* CameraSettings (Ray.hs:40-68) with the background reified. */
typedef struct rt_camera_settings {
  double center[3];
  double look_at[3];
  double up[3];
  double vfov;              /* radians */
  double aspect_ratio;
  int32_t image_width;
  int32_t samples_per_pixel;
  int32_t max_recursion_depth;
  int32_t background_kind;  /* RT_BG_* */
  double background_c0[3];
  double background_c1[3];
  double defocus_angle;     /* radians */
  double focus_dist;
  int32_t n_redirect_targets;
  int32_t pad;
  const rt_redirect_target* redirect_targets;
} rt_camera_settings;

/* rt_exec.flags (any other bit, or both RT_EXEC_ENCODE8_* bits, is RT_E_INVALID) */
#define RT_EXEC_F32 1          /* FP32 kernel, float output (default: binary64, double output) */
/* 8-bit output (rt_render / rt_multi_render only): out_rgb receives uint8 codes, one per channel,
   exactly what writeImage (sRGB) / writeImageSqrt (sqrt) store (Ray.hs:248-260):
   min(255, floor(256 * transfer(clamp01 x))) of the linear mean, NaN -> 0 — the fused epilogue
   of rt_encode8_async, run on the gathering device after the gather.  Bit-identical to encoding
   the linear render on the host. */
#define RT_EXEC_ENCODE8_SRGB 2
#define RT_EXEC_ENCODE8_SQRT 4
/* rt_render_async only: this render does not overlap another on the device (one stream, or the
   caller waits for it), so its work is planned for a short end, as rt_render's: 16-sample big
   items instead of up to 64 (rt_build.cpp rt_host_plan_work).  Images are identical either way. */
#define RT_EXEC_SOLO 8

#define RT_MAX_DEVICES 64

/* Which rows this call renders, on which devices, in which precision.
 *
 * Rows are dealt to shards in blocks of `row_block` round-robin: shard r owns global rows y
 * with (y / row_block) % n_shards == r.  With n_shards > 1 every shard has the same padded row
 * count (rt_shard_rows); padding rows are written as zeros.  With n_shards == 1 the tile is
 * exactly the image (height rows).  This is the one-process-per-GPU form (each rank renders
 * its shard on `device`).
 *
 * Device list (rt_render only; one process, many GPUs).  With n_devices >= 1 and n_shards == 1
 * the call renders the WHOLE image over devices[0 .. n_devices-1]: device k renders shard k of
 * n_devices (same row interleave), all devices concurrently on their own streams.  The scene is
 * built on the host ONCE and uploaded to the distinct devices concurrently; each device copies its
 * tile into devices[0]'s framebuffer (peer-to-peer over xGMI, the rows un-permuted by the copy's
 * stride), and one device-to-host copy fills out_rgb.  A device may appear more than once (two
 * shards on one GPU).  The image is bit-identical to the single-device render.  n_devices == 0:
 * `device` alone.  rt_multi_scene_create keeps such a scene resident across renders. */
typedef struct rt_exec {
  int32_t device;       /* HIP device ordinal (n_devices == 0) */
  int32_t n_shards;     /* >= 1 */
  int32_t shard;        /* 0 .. n_shards-1 */
  int32_t row_block;    /* >= 1 */
  int32_t flags;        /* RT_EXEC_* */
  int32_t n_devices;    /* 0, or 1 .. RT_MAX_DEVICES entries of `devices` (rt_render only) */
  const int32_t* devices;
} rt_exec;

typedef struct rt_stats {
  double upload_ms;     /* scene build + host->device copy (all devices) */
  double kernel_ms;     /* device time of the render (the slowest device of a device list) */
  double total_ms;      /* wall time of the call */
  int64_t samples;      /* pixels x spp rendered by this call */
  int32_t bvh_nodes;    /* nodes of all sets */
  int32_t max_stack;    /* deepest traversal stack the build can require */
  int32_t device_allocs; /* device allocations (hipMalloc) this call made: a resident multi-device
                            scene allocates its buffers on its first render (or a larger frame)
                            only, so later rt_multi_render calls report 0 (ABI v5) */
  int32_t kernel_block; /* workgroup size of the render kernel the call launched (ABI v6; the
                           1024-lane BVH classes run a 512-lane twin for a BVH whose traversal
                           stacks do not fit one 1024-lane workgroup's LDS); 0 from rt_scene_stats */
} rt_stats;

typedef struct rt_device_scene rt_device_scene;   /* opaque, device-resident scene */
typedef struct rt_multi_scene rt_multi_scene;     /* opaque, resident on a list of devices */

int rt_abi_version(void);
const char* rt_last_error(void);   /* thread-local message of the last failing call */
/* number of visible HIP devices (>= 1), or RT_E_HIP when there is none — what a caller puts in a
 * device list to render on every GPU of the node (rt_exec.devices) */
int rt_device_count(void);

/* image height for a width and aspect ratio: round (w / aspect), banker's rounding (Ray.hs:123) */
int rt_image_height(const rt_camera_settings* cs);
/* padded rows per shard for an image of `height` rows under `ex` */
int rt_shard_rows(int32_t height, const rt_exec* ex);
/* global row of shard-local row t (may be >= height for padding rows) */
int rt_shard_row(int32_t t, const rt_exec* ex);

/* One-shot host-buffer call — the Haskell binding's entry point (replaces Ray.hs:121-238).
 * out_rgb: caller-owned host buffer of rt_shard_rows(h, ex) * image_width * 3 doubles (floats
 * with RT_EXEC_F32, uint8 codes with RT_EXEC_ENCODE8_*); the whole image when n_shards == 1.  Returns RT_OK or a negative RT_E_*
 * code.  On RT_E_STACK a one-device call has written the partial image to out_rgb (a device list
 * leaves it untouched); the caller renders such a scene on the CPU path.  No copy into out_rgb is
 * in flight once the call has returned, whatever the code. */
int rt_render(const rt_camera_settings* cs, const rt_scene* scene, uint64_t seed, const rt_exec* ex,
              void* out_rgb, rt_stats* stats);

/* Device-resident path (used when inputs already live in HBM, e.g. bench.py / torch callers).
 * The scene is built on the host at create; a precision's records are uploaded on its first
 * render (rt_stats.upload_ms of rt_scene_stats covers what has been uploaded so far).  That first
 * render of a precision is therefore NOT asynchronous: it makes synchronous device allocations and
 * copies (and queries the kernel's occupancy) before it enqueues; a caller that captures the
 * stream into a HIP graph, or needs the first call to return at once, renders that precision
 * once beforehand. */
int rt_scene_create(const rt_scene* scene, int32_t device, rt_device_scene** out);
int rt_scene_destroy(rt_device_scene* s);
int rt_scene_stats(const rt_device_scene* s, rt_stats* stats);
/* Enqueue one render on `hip_stream` (a hipStream_t, or NULL for the default stream) of the
 * scene's device.  d_out_rgb: device buffer of rt_shard_rows(h, ex) * image_width * 3 doubles
 * (floats with RT_EXEC_F32).  ex->n_devices must be 0.  Asynchronous; the scene must outlive
 * the work.  Renders are planned for frames that overlap on two or more streams (the next frame
 * fills the end of this one); RT_EXEC_SOLO plans a render that runs alone. */
int rt_render_async(const rt_device_scene* s, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex,
                    void* d_out_rgb, void* hip_stream);

/* Multi-device resident scene (one process, many GPUs; what a caller that renders the same scene
 * more than once keeps between rt_render-like calls): one host build, concurrent uploads to the
 * distinct devices of the list, and per device its tile, render workspace, stream and events plus
 * the first device's gather and 8-bit buffers, all kept across renders (allocated on the first
 * render, or again for a larger frame: rt_stats.device_allocs).  Renders of one scene are
 * serialised (a mutex); the status word (traversal-stack overflow) is cleared before each.  rt_multi_render renders as rt_render does with this device list
 * (ex->n_devices must be 0; ex->n_shards 1, row_block and flags as in rt_render) into the
 * caller's host buffer out_rgb (h * width * 3 doubles, floats with RT_EXEC_F32, bytes with
 * RT_EXEC_ENCODE8_*).  A list of one device also renders an rt_exec shard (n_shards > 1). */
int rt_multi_scene_create(const rt_scene* scene, const int32_t* devices, int32_t n_devices, rt_multi_scene** out);
int rt_multi_scene_destroy(rt_multi_scene* m);
int rt_multi_render(const rt_multi_scene* m, const rt_camera_settings* cs, uint64_t seed, const rt_exec* ex,
                    void* out_rgb, rt_stats* stats);

/* Fused output epilogue of writeImage / writeImageSqrt (Ray.hs:248-260): linear RGB (float, or
 * double with in_f64 = 1) -> 8-bit codes min(255, floor(256 * transfer(clamp01 x))), transfer =
 * sRGB (encoding 0) or sqrt (encoding 1), evaluated in binary64; NaN -> 0.  Bit-exact against
 * the host encoder.  Device pointers, asynchronous on hip_stream. */
int rt_encode8_async(const void* d_rgb, int32_t in_f64, uint8_t* d_out, int64_t n_values, int32_t encoding,
                     void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* RT_AMD_H */
