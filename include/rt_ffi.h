/*
 * rt_ffi.h — C ABI of the MI355X-native path-tracing render kernel.
 *
 * Drop-in boundary for the per-pixel sample loop of SuneelFreimuth/raytracer-server. Each entry
 * point names the reference interface it replaces (paths relative to the reference repo root):
 *
 *   rt_scene_load_toml  <- Scene::from_toml                  src/scene.rs:143-150 (+ SceneSpec::to_scene :357-441)
 *   rt_scene_create     <- Scene::new + Mesh::accelerate     src/scene.rs:126-141, src/geometry.rs:835-837
 *                          (for a host that keeps its own loader and hands over flattened objects)
 *   rt_render           <- RenderJob::run's per-pixel loop   src/server.rs:157-199 calling
 *                          sample_pixel + gamma_correct      src/server.rs:320-368 (and the `as u8` at :187-189)
 *   rt_render_device    <- same, device-resident output, enqueued on a caller HIP stream (no host sync)
 *   rt_render_multi     <- same, bands handed out dynamically to several devices (the row-band fan-out of
 *                          RenderJob::run, server.rs:165-168), host gather
 *   rt_trace_rays       <- Scene::trace_ray                  src/scene.rs:272-289 (batch form, for parity tests)
 *
 * Conventions (mirroring the reference's):
 *   - a scene is immutable after creation and may be shared by concurrent rt_render calls
 *     (the reference shares Arc<HashMap<String, Scene>>, server.rs:24);
 *   - errors never abort: every call returns RT_OK (0), RT_CANCELLED (1) or a negative RT_E_*
 *     code, and rt_last_error() gives a thread-local message (the reference panics instead);
 *   - images are row-major RGB8, row 0 = top; pixel (x, row) is the reference's
 *     sample_pixel(x, height - row - 1, ...) (server.rs:179-186);
 *   - spp follows the reference: 4 * floor(spp / 4) samples are traced (server.rs:332); spp < 4
 *     renders black exactly like the reference.
 *   - randomness: counter-based, one stream per camera sample: Philox4x32-10 keyed by the seed, with
 *     counter (global pixel, sample, 0, subpixel), seeds an xoroshiro128++ stream that the path consumes
 *     in the reference's draw order; output is independent of tiling, device count and
 *     kernel mode.
 */
#ifndef RT_FFI_H
#define RT_FFI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3  /* 2: rt_render_params.row_step; 3: rt_render_multi */

/* return codes */
#define RT_OK 0
#define RT_CANCELLED 1
#define RT_E_INVAL (-1)
#define RT_E_HIP (-2)
#define RT_E_OOM (-3)
#define RT_E_IO (-4)
#define RT_E_PARSE (-5)
#define RT_E_NODEVICE (-6)

/* rt_render_params.flags */
#define RT_FLAG_MIS (1u << 0)        /* config.toml `use_mis` (dead in the reference, scene.rs:188): build-defined balance heuristic */
#define RT_FLAG_MEGAKERNEL (1u << 1) /* fused per-lane path loop instead of the wavefront pipeline */
#define RT_FLAG_FP32 (1u << 2)       /* f32 perf mode (statistical parity only): diffuse/mirror BRDFs and
                                        sphere lights (RT_E_INVAL otherwise), meshes with nearest-triangle semantics;
                                        implies the megakernel. Default is the reference's f64 */
#define RT_FLAG_MESH_NEAREST (1u << 3) /* Mesh::intersect's `octree: None` branch (geometry.rs:886-903: nearest
                                          triangle, strict < in index order) instead of the octree walk, accelerated on
                                          the device by a BVH; megakernel only (RT_E_INVAL with the wavefront) */

typedef struct rt_scene rt_scene;

enum { RT_BRDF_DIFFUSE = 0, RT_BRDF_SPECULAR = 1, RT_BRDF_PHONG = 2 };   /* scene.rs:18-28 */
enum { RT_GEOM_SPHERE = 0, RT_GEOM_PLANE = 1, RT_GEOM_MESH = 2 };       /* geometry.rs:388-392 */

typedef struct {
    double emitted[3];          /* Object.emitted (scene.rs:12) */
    int32_t brdf_kind;          /* RT_BRDF_* */
    double k[3];                /* Diffuse kd / Specular ks */
    double phong_kd, phong_ks;  /* Phong (scene.rs:21-27) */
    int32_t phong_power;
    double color_d[3], color_s[3];
    int32_t geom_kind;          /* RT_GEOM_* */
    double pos[3];              /* sphere centre / plane point */
    double r;                   /* sphere radius */
    double n[3];                /* plane normal */
    int32_t mesh;               /* index into rt_scene_desc.meshes (RT_GEOM_MESH) */
} rt_object_desc;

typedef struct {
    uint32_t n_vertices;
    const double* vertices;     /* 3 per vertex, after transforms (geometry.rs:427-510) */
    uint32_t n_triangles;
    const uint32_t* indices;    /* 3 per triangle (0-based) */
    double bbox_min[3];         /* Mesh.bounding_box exactly as the reference holds it after */
    double bbox_max[3];         /*   transforms (octree root box, geometry.rs:1153) */
    double surface_area;        /* Mesh.surface_area (geometry.rs:771; mesh-light pdf) */
} rt_mesh_desc;

typedef struct {
    double cam_pos[3], cam_dir[3];   /* Scene.camera (scene.rs:104) */
    uint32_t n_objects;
    const rt_object_desc* objects;
    uint32_t n_meshes;
    const rt_mesh_desc* meshes;
} rt_scene_desc;

typedef struct {
    int32_t width, height;       /* full image (camera frame uses these, server.rs:328-331) */
    int32_t x0, y0;              /* tile origin, screen coordinates (row 0 = top) */
    int32_t tile_w, tile_h;      /* tile size; output buffers are tile_w * tile_h pixels */
    int32_t spp;                 /* reference semantics (server.rs:332) */
    uint64_t seed;
    uint32_t flags;              /* RT_FLAG_* */
    int32_t device;              /* HIP device ordinal */
    int32_t row_step;            /* tile row i is screen row y0 + i * row_step (0 or 1: contiguous rows);
                                    k > 1 interleaves rows across k workers (multi-GPU load balance) */
} rt_render_params;

typedef struct {
    int64_t samples;             /* camera samples traced = tile pixels * 4 * floor(spp/4) */
    int64_t vertices;            /* path vertices (extension rays that hit) */
    int64_t iterations;          /* wavefront bounce iterations (0 for the megakernel) */
    double device_ms;            /* device time of the render (HIP events on the render stream) */
    double kernel_ms[8];         /* per-stage device time (wavefront: extend, shade, shadow, regen, finalize) */
    int64_t kernel_launches[8];
} rt_render_stats;

/* Scene construction ---------------------------------------------------------------------- */
int rt_scene_load_toml(const char* toml_path, const char* assets_dir /* NULL: <toml dir>/assets */, rt_scene** out);
int rt_scene_create(const rt_scene_desc* desc, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);

/* Scene inspection (host prep parity: octree shape etc.). info[16] int64:
 * [0]=objects [1]=light index [2]=meshes [3]=total octree nodes [4]=parents [5]=leaves
 * [6]=triangle refs [7]=triangles [8]=vertices [9]=max leaf size [10]=max leaf depth
 * [11]=1 if the octree walks use the child-slot tables (subtree culls), 0 if they read the plain child
 * tables (octrees whose node ids exceed the slot encoding, 2^23; same results either way) */
int rt_scene_info(const rt_scene* scene, int64_t info[16]);
/* Per-object mesh data after transforms: bbox[6], surface area, octree in DFS pre-order
 * (kind: 0 parent/1 leaf, child[8*n], leaf_off, leaf_cnt, refs). Any output pointer may be NULL. */
int rt_scene_mesh(const rt_scene* scene, int32_t object, int64_t counts[4] /* nodes, refs, tris, verts */,
                  double bbox[6], double* surface_area, double* vertices, uint32_t* indices,
                  int32_t* kind, int32_t* child, int32_t* leaf_off, int32_t* leaf_cnt, int32_t* refs);

/* Rendering ------------------------------------------------------------------------------- */
/* Host buffers: rgb_out tile_w*tile_h*3 u8; sub_out (optional) tile_w*tile_h*4*3 f64 subpixel
 * means before the clamp; cancel (optional; nonzero = stop, returns RT_CANCELLED): read by the
 * calling thread while the render runs and copied into a pinned word the megakernels poll between
 * subpixels (the wavefront: between bounce batches). The flag is never registered with HIP and may be
 * shared by concurrent renders. stats optional. */
int rt_render(const rt_scene* scene, const rt_render_params* params, uint8_t* rgb_out, double* sub_out,
              const volatile int32_t* cancel, rt_render_stats* stats);
/* Device buffers on params->device; enqueued on `stream` (hipStream_t, NULL = default stream).
 * Synchronous with respect to the stream only when stats != NULL. */
int rt_render_device(const rt_scene* scene, const rt_render_params* params, void* d_rgb, void* d_sub,
                     void* stream, rt_render_stats* stats);

/* One process, several devices (replaces the row-band fan-out of RenderJob::run,
 * server.rs:165-168): the tile's rows are cut into bands of `band_rows` tile rows (<= 0: about 8 bands per
 * worker) handed out dynamically from a host atomic counter to one worker thread per entry of `devices`
 * (an ordinal may repeat: several workers on one device). A worker renders each band with the device path on
 * its own streams (two bands in flight, so one band's tail overlaps the next band's start) and copies the RGB8
 * rows straight into rgb_out: the gather is host-side, no collective. The image is byte-identical to rt_render
 * of the same params (the RNG is keyed by global pixel). cancel is checked between bands and relayed to
 * the running bands' kernels as in rt_render. stats (optional):
 * samples and vertices summed over the bands, device_ms = wall time of the whole call.
 * Errors, checked before any band runs: RT_E_NODEVICE when no HIP device is visible (or the runtime is
 * absent), RT_E_INVAL for a device ordinal outside [0, device count). */
int rt_render_multi(const rt_scene* scene, const rt_render_params* params, const int32_t* devices, int32_t n_devices,
                    int32_t band_rows, uint8_t* rgb_out, const volatile int32_t* cancel, rt_render_stats* stats);
/* The band plan rt_render_multi hands out (no GPU): band b = tile rows [first_row[b], first_row[b] + rows[b]),
 * in handout order. Returns the band count; writes at most `cap` entries (either array may be NULL). */
int32_t rt_band_plan(int32_t tile_h, int32_t n_workers, int32_t band_rows, int32_t cap, int32_t* first_row,
                     int32_t* rows);

/* Scene::trace_ray on the device for n host rays: t, object id (-1: no hit), hit pos/normal. */
int rt_trace_rays(const rt_scene* scene, int32_t device, int64_t n, const double* origins, const double* dirs,
                  double* t, int32_t* object, double* pos, double* normal);
/* The same with render flags (RT_FLAG_MESH_NEAREST selects the nearest-triangle mesh semantics). */
int rt_trace_rays_flags(const rt_scene* scene, int32_t device, uint32_t flags, int64_t n, const double* origins,
                        const double* dirs, double* t, int32_t* object, double* pos, double* normal);

const char* rt_last_error(void);
int rt_abi_version(void);
int rt_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_FFI_H */
