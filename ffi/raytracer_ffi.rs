//! Rust bindings of the MI355X render kernel's C ABI (`include/rt_ffi.h`, ABI version 3), for the
//! reference host (SuneelFreimuth/raytracer-server). A maintainer adds this file as
//! `src/raytracer_ffi.rs` and links `librtamd.so` (`raytracer-server_amd/lib/`, built by
//! `make -C raytracer-server_amd`), e.g. from `build.rs`:
//!
//! ```ignore
//! println!("cargo:rustc-link-search=native=/path/to/raytracer-server_amd/lib");
//! println!("cargo:rustc-link-lib=dylib=rtamd");
//! ```
//!
//! Not compiled in this repository (no Rust toolchain in the build image); the declarations mirror
//! `rt_ffi.h` field for field, and `tests/test_abi.py` checks that header's struct layouts and
//! exported symbols. What each entry point replaces in the reference:
//!
//! | entry point          | reference                                                              |
//! |----------------------|------------------------------------------------------------------------|
//! | `rt_scene_load_toml` | `Scene::from_toml` (src/scene.rs:143-150, `SceneSpec::to_scene` :357-441) |
//! | `rt_scene_create`    | `Scene::new` + `Mesh::accelerate` (src/scene.rs:126-141, src/geometry.rs:835-837) |
//! | `rt_render`          | `RenderJob::run`'s per-pixel loop (src/server.rs:157-199) over `sample_pixel` + `gamma_correct` (:320-368) |
//! | `rt_render_device`   | the same, device-resident output on a caller HIP stream                |
//! | `rt_render_multi`    | the row-band fan-out of `RenderJob::run` (src/server.rs:165-168) over several GPUs |
//! | `rt_trace_rays`      | `Scene::trace_ray` (src/scene.rs:272-289), batch form                  |
//!
//! Conventions: a scene is immutable after creation and may be shared by concurrent renders (the
//! reference's `Arc<HashMap<String, Scene>>`, src/server.rs:24); errors are return codes (`RT_OK`,
//! `RT_CANCELLED`, negative `RT_E_*`) with a thread-local message from `rt_last_error`; images are
//! row-major RGB8 with row 0 at the top (the `height - y - 1` flip of src/server.rs:181); `spp`
//! keeps the reference's `spp / 4` samples per subpixel (src/server.rs:332).

#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

pub const RT_ABI_VERSION: c_int = 3;

pub const RT_OK: c_int = 0;
pub const RT_CANCELLED: c_int = 1;
pub const RT_E_INVAL: c_int = -1;
pub const RT_E_HIP: c_int = -2;
pub const RT_E_OOM: c_int = -3;
pub const RT_E_IO: c_int = -4;
pub const RT_E_PARSE: c_int = -5;
pub const RT_E_NODEVICE: c_int = -6;

/// `config.toml`'s `use_mis` (dead in the reference, src/scene.rs:188): build-defined balance heuristic.
pub const RT_FLAG_MIS: u32 = 1 << 0;
/// Fused per-lane path loop (the fast path) instead of the wavefront pipeline.
pub const RT_FLAG_MEGAKERNEL: u32 = 1 << 1;
/// f32 perf mode: statistical parity only; implies the megakernel.
pub const RT_FLAG_FP32: u32 = 1 << 2;
/// `Mesh::intersect` without the octree (src/geometry.rs:886-903), a BVH on the device.
pub const RT_FLAG_MESH_NEAREST: u32 = 1 << 3;

pub const RT_BRDF_DIFFUSE: i32 = 0;
pub const RT_BRDF_SPECULAR: i32 = 1;
pub const RT_BRDF_PHONG: i32 = 2;
pub const RT_GEOM_SPHERE: i32 = 0;
pub const RT_GEOM_PLANE: i32 = 1;
pub const RT_GEOM_MESH: i32 = 2;

/// Opaque scene handle (`rt_scene`).
#[repr(C)]
pub struct RtScene {
    _private: [u8; 0],
}

/// `rt_object_desc`: one reference `Object` (src/scene.rs:10-15) with its BRDF and geometry flattened.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RtObjectDesc {
    pub emitted: [f64; 3],
    pub brdf_kind: i32,
    pub k: [f64; 3],
    pub phong_kd: f64,
    pub phong_ks: f64,
    pub phong_power: i32,
    pub color_d: [f64; 3],
    pub color_s: [f64; 3],
    pub geom_kind: i32,
    pub pos: [f64; 3],
    pub r: f64,
    pub n: [f64; 3],
    pub mesh: i32,
}

/// `rt_mesh_desc`: a mesh after its transforms (src/geometry.rs:427-510); `bbox_*` as the reference
/// holds `Mesh.bounding_box` (the octree root box, src/geometry.rs:1153).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct RtMeshDesc {
    pub n_vertices: u32,
    pub vertices: *const f64,
    pub n_triangles: u32,
    pub indices: *const u32,
    pub bbox_min: [f64; 3],
    pub bbox_max: [f64; 3],
    pub surface_area: f64,
}

/// `rt_scene_desc`: camera (src/scene.rs:104) plus flattened objects and meshes.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct RtSceneDesc {
    pub cam_pos: [f64; 3],
    pub cam_dir: [f64; 3],
    pub n_objects: u32,
    pub objects: *const RtObjectDesc,
    pub n_meshes: u32,
    pub meshes: *const RtMeshDesc,
}

/// `rt_render_params`: a tile of a `width x height` frame (screen rows, row 0 = top).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RtRenderParams {
    pub width: i32,
    pub height: i32,
    pub x0: i32,
    pub y0: i32,
    pub tile_w: i32,
    pub tile_h: i32,
    pub spp: i32,
    pub seed: u64,
    pub flags: u32,
    pub device: i32,
    /// 0 or 1: contiguous tile rows; k > 1: tile row i is screen row y0 + i * k.
    pub row_step: i32,
}

/// `rt_render_stats`.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct RtRenderStats {
    pub samples: i64,
    pub vertices: i64,
    pub iterations: i64,
    pub device_ms: f64,
    pub kernel_ms: [f64; 8],
    pub kernel_launches: [i64; 8],
}

extern "C" {
    pub fn rt_scene_load_toml(toml_path: *const c_char, assets_dir: *const c_char, out: *mut *mut RtScene) -> c_int;
    pub fn rt_scene_create(desc: *const RtSceneDesc, out: *mut *mut RtScene) -> c_int;
    pub fn rt_scene_destroy(scene: *mut RtScene);
    pub fn rt_scene_info(scene: *const RtScene, info: *mut i64 /* [16] */) -> c_int;
    pub fn rt_scene_mesh(
        scene: *const RtScene, object: i32, counts: *mut i64 /* [4] */, bbox: *mut f64 /* [6] */,
        surface_area: *mut f64, vertices: *mut f64, indices: *mut u32, kind: *mut i32, child: *mut i32,
        leaf_off: *mut i32, leaf_cnt: *mut i32, refs: *mut i32,
    ) -> c_int;

    /// Host buffers: `rgb_out` tile_w * tile_h * 3 bytes; `sub_out` (nullable) tile_w * tile_h * 12
    /// f64 subpixel means before the clamp. `cancel` (nullable): the job's `AtomicBool`
    /// (src/server.rs:226-251) viewed as an `i32`, read while the render runs; it may be shared by
    /// concurrent renders and is never registered with HIP. Returns `RT_CANCELLED` when it stopped
    /// the render.
    pub fn rt_render(
        scene: *const RtScene, params: *const RtRenderParams, rgb_out: *mut u8, sub_out: *mut f64,
        cancel: *const i32, stats: *mut RtRenderStats,
    ) -> c_int;
    /// Device buffers on `params.device`, enqueued on `stream` (a `hipStream_t`, null = default
    /// stream); synchronous with respect to the stream only when `stats` is non-null.
    pub fn rt_render_device(
        scene: *const RtScene, params: *const RtRenderParams, d_rgb: *mut c_void, d_sub: *mut c_void,
        stream: *mut c_void, stats: *mut RtRenderStats,
    ) -> c_int;
    /// Several devices (one worker thread per entry of `devices`; ordinals may repeat), bands of
    /// `band_rows` rows (<= 0: about 8 per worker) handed out dynamically, host gather into `rgb_out`.
    pub fn rt_render_multi(
        scene: *const RtScene, params: *const RtRenderParams, devices: *const i32, n_devices: i32,
        band_rows: i32, rgb_out: *mut u8, cancel: *const i32, stats: *mut RtRenderStats,
    ) -> c_int;
    /// The band plan of `rt_render_multi` (no GPU); returns the band count, writes at most `cap`.
    pub fn rt_band_plan(
        tile_h: i32, n_workers: i32, band_rows: i32, cap: i32, first_row: *mut i32, rows: *mut i32,
    ) -> i32;

    pub fn rt_trace_rays(
        scene: *const RtScene, device: i32, n: i64, origins: *const f64, dirs: *const f64, t: *mut f64,
        object: *mut i32, pos: *mut f64, normal: *mut f64,
    ) -> c_int;
    pub fn rt_trace_rays_flags(
        scene: *const RtScene, device: i32, flags: u32, n: i64, origins: *const f64, dirs: *const f64,
        t: *mut f64, object: *mut i32, pos: *mut f64, normal: *mut f64,
    ) -> c_int;

    pub fn rt_last_error() -> *const c_char;
    pub fn rt_abi_version() -> c_int;
    pub fn rt_device_count() -> c_int;
}

/// Owned scene handle: destroyed on drop; `Send + Sync` because the library allows concurrent
/// renders on one scene (rt_ffi.h), like the reference's shared `Arc<Scene>`.
pub struct Scene(pub *mut RtScene);
unsafe impl Send for Scene {}
unsafe impl Sync for Scene {}
impl Drop for Scene {
    fn drop(&mut self) {
        unsafe { rt_scene_destroy(self.0) }
    }
}

/// The library's last error on this thread.
pub fn last_error() -> String {
    unsafe {
        let p = rt_last_error();
        if p.is_null() {
            String::new()
        } else {
            std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    }
}

/// Loads a scene the way `Scene::from_toml` does (meshes from `<toml dir>/assets`).
pub fn load_scene(toml_path: &str) -> Result<Scene, String> {
    let path = std::ffi::CString::new(toml_path).map_err(|e| e.to_string())?;
    let mut s: *mut RtScene = std::ptr::null_mut();
    let rc = unsafe { rt_scene_load_toml(path.as_ptr(), std::ptr::null(), &mut s) };
    if rc == RT_OK {
        Ok(Scene(s))
    } else {
        Err(format!("rt_scene_load_toml: {} ({})", rc, last_error()))
    }
}

/// `RenderJob::run`'s frame (src/server.rs:157-199) in one call: the RGB8 frame, or `None` when the
/// job was cancelled. `cancel` is the job's stop flag kept as an `AtomicI32` (the reference's
/// `AtomicBool`, src/server.rs:226-251; `stop()` stores 1); it is read while the render runs. The caller
/// then emits the reference's chunk messages per screen row `y` and 60-pixel window `x`
/// (src/server.rs:169-192): `[0u8, n as u8, x as u16 LE, y as u16 LE]` followed by
/// `rgb[(y * width + x) * 3 ..][.. 3 * n]`. Call it from `tokio::task::spawn_blocking`.
pub fn render_frame(
    scene: &Scene, width: i32, height: i32, spp: i32, seed: u64, cancel: &std::sync::atomic::AtomicI32,
) -> Result<Option<Vec<u8>>, String> {
    let p = RtRenderParams {
        width, height, x0: 0, y0: 0, tile_w: width, tile_h: height, spp, seed,
        flags: RT_FLAG_MEGAKERNEL, device: 0, row_step: 1,
    };
    let mut rgb = vec![0u8; (width as usize) * (height as usize) * 3];
    let rc = unsafe {
        rt_render(scene.0, &p, rgb.as_mut_ptr(), std::ptr::null_mut(), cancel.as_ptr() as *const i32,
                  std::ptr::null_mut())
    };
    match rc {
        RT_OK => Ok(Some(rgb)),
        RT_CANCELLED => Ok(None),
        _ => Err(format!("rt_render: {} ({})", rc, last_error())),
    }
}
