/*
 * mi355r — MI355X-native differentiable mesh rasterizer: public C ABI.
 *
 * Plain pointers + sizes, no torch types. All device pointers live in HBM of
 * the current HIP device; every call is asynchronous on `stream` (a
 * hipStream_t passed as void*) and performs no host synchronisation and no
 * device allocation: callers own outputs and workspace (sized with the
 * *_workspace() queries). Returns MR_OK (0) or an error code; the message is
 * in mr_last_error() (thread-local).
 *
 * Boundary being replaced (reference path: torch_renderer.py:97-159,
 * renderer.py:87-101 -> PyTorch3D MeshRasterizer/MeshRenderer ->
 * pybind11 module pytorch3d._C, upstream csrc/ext.cpp):
 *   _C.rasterize_meshes           -> mr_rasterize_meshes
 *   _C.rasterize_meshes_backward  -> mr_rasterize_meshes_backward
 *   MeshRasterizer.transform (torch bmm) -> mr_project_faces(+_backward)
 *   SoftPhongShader + SoftSilhouetteShader + zbuf relu over ONE raster pass
 *     (torch_renderer.py:110-121 rasterizes twice; :155-159 once more)
 *                                -> mr_render_forward / mr_render_backward
 */
#ifndef MI355R_H
#define MI355R_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MR_OK = 0, MR_EINVAL = 1, MR_ELAUNCH = 2, MR_EUNSUPPORTED = 3, MR_EWORKSPACE = 4 };

/* Per-view camera: X_view = X_world @ R + T (PyTorch3D row-vector
 * convention, R row-major), ndc = (ax * x/z + bx, ay * y/z + by, z).
 * PerspectiveCameras(in_ndc=False): ax = fx/s, bx = (W/2 - px)/s, s = min(H,W)/2
 * (torch_renderer.py:61-71); FoVPerspectiveCameras: ax = 1/(tan(fov/2)*aspect).
 * 64 bytes. */
typedef struct mr_view {
  float R[9];
  float T[3];
  float ax, bx, ay, by;
} mr_view_t;

/* RasterizationSettings (upstream rasterizer.py) — blur/K/clip/cull as there. */
typedef struct mr_raster_settings {
  int32_t H, W;
  int32_t faces_per_pixel;   /* 1..128 on mr_rasterize_meshes; 1 on the fused mr_render_* path */
  float blur_radius;
  int32_t perspective_correct;
  int32_t clip_barycentric_coords;
  int32_t cull_backfaces;
  int32_t max_faces_per_bin; /* <= 0: library default; overflow is handled exactly */
  /* Near-plane clipping (upstream MeshRasterizer: z_clip_value = znear / 2 for FoVPerspectiveCameras,
   * then mesh/clip.py clip_faces -> rasterize -> convert_clipped_rasterization_to_original_faces).
   * clip_z != 0: faces crossing view z = z_clip_value are split (one or two sub-triangles, the two
   * halves of a clipped quadrilateral being each other's clipped_faces_neighbor_idx); outputs refer
   * to the original faces (pix_to_face, barycentrics converted back); backward chains through the
   * split. Done inside the binning kernels: no host round trip, nothing to do when nothing crosses. */
  int32_t clip_z;
  float z_clip_value;
} mr_raster_settings_t;

/* Shading / blending parameters (SoftPhongShader, PointLights, Materials,
 * BlendParams, SoftSilhouetteShader). */
typedef struct mr_shade_params {
  int32_t light_kind;        /* 0 = PointLights, 1 = AmbientLights */
  float light_location[3];
  float light_ambient[3], light_diffuse[3], light_specular[3];
  float mat_ambient[3], mat_diffuse[3], mat_specular[3];
  float shininess;
  float sigma_rgb, gamma, background[3], znear, zfar;
  float sigma_sil;
  int32_t out_flags;         /* MR_OUT_* */
  int32_t rgb_channels;      /* 3 (rgb) or 4 (rgba, alpha = 1 - prod(1 - prob)) */
} mr_shade_params_t;

enum { MR_OUT_DEPTH = 1, MR_OUT_SIL = 2, MR_OUT_RGB = 4,
       /* with MR_OUT_RGB, mr_shade_fragments_* only: upstream hard_rgb_blend (HardPhongShader) —
        * the nearest fragment's Phong colour or the background, alpha = 1 where a face covers the
        * pixel; gradients reach the colour of the nearest fragment only */
       MR_OUT_HARD = 8,
       /* mr_render_backward[_opencv] only: the forward workspace's per-face gradient totals are as the
        * forward left them (cleared), i.e. this is the first backward over that forward; the
        * backward then skips clearing them. Leave it unset for any later backward over the same
        * forward workspace (e.g. autograd retain_graph). */
       MR_GRAD_ROWS_CLEARED = 16,
       /* with MR_OUT_SIL, mr_render_forward/_backward[_opencv]: the silhouette buffer is (N,H,W,4)
        * RGBA as SoftSilhouetteShader returns it, (1, 1, 1, alpha) per pixel, written by the
        * kernels; its gradient is the (N,H,W,4) gradient of that tensor (channel 3 is read) */
       MR_OUT_SIL_RGBA = 32,
       /* with MR_OUT_DEPTH, mr_render_forward/_backward[_opencv]: the depth buffer is MeshRasterizer's
        * zbuf[..., 0] of K = 1 fragments (the nearest face's depth, -1 where no face) instead of
        * DepthRender's relu of it (camera_pose_optimizer.py:244-246 reads rasterizer(...).zbuf). */
       MR_OUT_ZBUF = 64,
       /* bits 8-9 (MR_SREC_SLOT(k), k < 4), mr_render_forward / _reshade / _backward: which of the forward
        * workspace's four per-face shading-record sets this call packs and its backward reads (0 for a
        * plain forward; mr_render_reshade calls sharing one workspace take distinct slots) */
       MR_SREC_SLOT_SHIFT = 8,
       /* mr_shade_fragments_* only: every pixel's empty slots (pix_to_face = -1) follow its filled
        * ones, as mr_rasterize_meshes[_world] (and PyTorch3D's rasterizer) write them; the kernels
        * then stop at a pixel's first empty slot instead of reading all K (same results).
        * Bit 10 since mr_version() 5 (it was 64, the value of MR_OUT_ZBUF, before). */
       MR_FRAG_SORTED = 1024 };

/* One triangle mesh shared by all N views (Meshes.extend(N)) — or, with
 * view_face_first set, a batch of N distinct meshes (renderer.py:78-80: N OBJ files in one Meshes),
 * view n rendering mesh n: the arrays then hold the meshes' union (each mesh's faces index its own
 * vertices inside the union; no vertex is shared between meshes). */
typedef struct mr_mesh {
  const float* verts;        /* (V,3) world */
  int64_t V;
  const int32_t* faces;      /* (F,3) */
  int64_t F;
  const int32_t* vadj_ptr;   /* (V+1) CSR vertex -> (face<<2 | corner), sorted by (corner, face) */
  const int32_t* vadj;
  const float* vnormals;     /* (V,3) from mr_vertex_normals (PointLights only) */
  int32_t tex_kind;          /* 0 white, 1 per-vertex colours, 2 UV map */
  const float* vcolors;      /* (V,3) */
  const float* verts_uvs;    /* (Vt,2) */
  const int32_t* faces_uvs;  /* (F,3) */
  const float* tex_rgba;     /* (Ht,Wt,4) float, image row 0 first (flip done in-kernel) */
  int32_t tex_h, tex_w;
  /* Optional (mr_render_forward only): when non-NULL the forward computes the vertex normals
   * itself into vnormals_out (V,3) and their un-normalised sums into vraw_out (V,3), in its first
   * launch, instead of reading `vnormals` (saves the separate mr_vertex_normals launch). */
  float* vnormals_out;
  float* vraw_out;
  /* Optional: the same map as 8-bit texels, (Ht,Wt,4) u8, when every value of tex_rgba is exactly
   * tex_lut[k] for some k (e.g. a PNG divided by 255): the samplers then read 4-B texels and
   * convert through the 256-entry table, bitwise the same values at a quarter of the bytes. */
  const uint8_t* tex_u8;
  const float* tex_lut;      /* (256) f32, required with tex_u8 */
  /* Distinct meshes (mr_render_*, mr_shade_fragments_*; NULL: one shared mesh). Device arrays:
   * view_face_first (N+1) the first union face of view n's mesh (view_face_first[N] = F) and
   * view_face_count (N) its face count; max_view_faces (host) = the largest count. Face ids stay
   * union face ids (= PyTorch3D's packed ids of the batch). Size the forward workspace with
   * mr_render_workspace_meshes. */
  const int64_t* view_face_first;
  const int64_t* view_face_count;
  int64_t max_view_faces;
} mr_mesh_t;

const char* mr_last_error(void);
int32_t mr_version(void);
/* sizeof of the ABI structs as compiled into the library (binding self-check):
 * 0 mr_view_t, 1 mr_raster_settings_t, 2 mr_shade_params_t, 3 mr_mesh_t; -1 otherwise. */
int32_t mr_struct_size(int32_t which);

/* ---------------- PyTorch3D _C.rasterize_meshes boundary ---------------- */
size_t mr_rasterize_meshes_workspace(int64_t num_meshes, int64_t total_faces, int32_t H, int32_t W,
                                     int32_t max_faces_per_bin);

/* face_verts (F,3,3) NDC xy + view z; mesh_to_face_first_idx / num_faces_per_mesh (N) int64 on device.
 * Outputs (N,H,W,K): pix_to_face int64 (packed face id or -1), zbuf, dists f32; bary (N,H,W,K,3). */
int32_t mr_rasterize_meshes(const float* face_verts, const int64_t* mesh_to_face_first_idx,
                            const int64_t* num_faces_per_mesh, int64_t num_meshes, int64_t total_faces,
                            const mr_raster_settings_t* settings, int64_t* pix_to_face, float* zbuf,
                            float* bary, float* dists, void* workspace, size_t workspace_bytes, void* stream);

/* Camera poses in the PyTorch3D convention (row-vector R (N,3,3), T (N,3); X_view = X_world R + T) with
 * the intrinsics rows {ax, bx, ay, by} (N,4) of mr_view_t; *_stride = floats between consecutive views
 * (0 broadcasts one row). Same layout as mr_opencv_poses_t. */
typedef struct mr_poses {
  const float* R;
  int64_t R_stride;
  const float* T;
  int64_t T_stride;
  const float* intr;
  int64_t intr_stride;
} mr_poses_t;

/* MeshRasterizer.forward for ONE mesh shared by N views (Meshes.extend; upstream
 * mesh/rasterizer.py transform + rasterize_meshes): verts (V,3) f32, faces (F,3) i32. Writes the
 * fragments (as mr_rasterize_meshes, packed face ids n*F + f), face_verts (N*F,3,3) — what
 * _RasterizeFaceVerts saves for mr_rasterize_meshes_backward, bitwise mr_project_faces' output — and
 * the view records views_out (N) for mr_project_faces_backward. The projection runs inside the
 * binning's first launch (no separate projection launch, no counter memset). */
size_t mr_rasterize_meshes_world_workspace(int64_t N, int64_t F, int32_t H, int32_t W, int32_t max_faces_per_bin);
int32_t mr_rasterize_meshes_world(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                  const mr_poses_t* poses, int64_t N, const mr_raster_settings_t* settings,
                                  mr_view_t* views_out, float* face_verts, int64_t* pix_to_face, float* zbuf,
                                  float* bary, float* dists, void* workspace, size_t workspace_bytes, void* stream);

/* Measurement helper (bench.py's per-kernel algorithmic bytes): output pixels whose background the
 * per-view binning launch (k_bin_view) writes on the CUs its view workgroups leave idle, for a
 * K = 1 forward of N views of F faces (mode 0: mr_rasterize_meshes[_world] fragments, 1: the
 * fused render); k_tile_raster writes the rest. */
int64_t mr_binning_background_pixels(int64_t N, int64_t F, int32_t H, int32_t W, int32_t mode);

/* grad_face_verts (F,3,3) is overwritten (zeroed then accumulated). Any of grad_zbuf, grad_bary,
 * grad_dists may be NULL (PyTorch passes None for an output the loss did not use): it counts as
 * zero, and no zero-filled tensor needs to be allocated for it. */
int32_t mr_rasterize_meshes_backward(const float* face_verts, const int64_t* pix_to_face,
                                     const float* grad_zbuf, const float* grad_bary, const float* grad_dists,
                                     int64_t num_meshes, int64_t total_faces, const mr_raster_settings_t* settings,
                                     float* grad_face_verts, void* stream);

/* ---------------- projection (MeshRasterizer.transform) ---------------- */
/* face_verts[n*F + f][c] = ndc(view n, verts[faces[f][c]]) for n < N. */
int32_t mr_project_faces(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                         const mr_view_t* views, int64_t N, float* face_verts, void* stream);
/* grad_verts (V,3) and grad_views (N,12: dR row-major, dT) are overwritten. */
int32_t mr_project_faces_backward(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                  const int32_t* vadj_ptr, const int32_t* vadj, const mr_view_t* views, int64_t N,
                                  const float* grad_face_verts, float* grad_verts, float* grad_views, void* stream);
/* The same for a batch of N distinct meshes (MeshRasterizer.transform of a Meshes of different
 * meshes, renderer.py:78-80): verts / faces are their union (see mr_mesh_t), view n projects only
 * mesh n's faces [view_face_first[n], view_face_first[n+1]) into face_verts rows of the same ids
 * (the packed order). The backward walks view n's own vertices [view_vert_first[n],
 * view_vert_first[n+1]); max_view_faces / max_view_verts are the largest per-mesh counts. */
int32_t mr_project_faces_meshes(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                const int64_t* view_face_first, int64_t max_view_faces, const mr_view_t* views,
                                int64_t N, float* face_verts, void* stream);
int32_t mr_project_faces_meshes_backward(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                         const int32_t* vadj_ptr, const int32_t* vadj, const int64_t* view_vert_first,
                                         int64_t max_view_verts, const mr_view_t* views, int64_t N,
                                         const float* grad_face_verts, float* grad_verts, float* grad_views,
                                         void* stream);

/* ---------------- camera poses (DifferentiableRenderer._camera_pose_from_opencv_to_pytorch) ---------------- */
/* torch_renderer.py:73-80: R_p3d = R_cv^T with columns 0,1 negated; T = t_cv with entries 0,1 negated.
 * views[n] = {R_p3d row-major, T, intr[n]} (bitwise what the torch conversion + packing gives).
 * *_stride = elements between consecutive views (0 broadcasts one pose / one intrinsics row). */
int32_t mr_views_from_opencv(const float* R_cv, int64_t R_stride, const float* t_cv, int64_t t_stride,
                             const float* intr, int64_t intr_stride, int64_t N, mr_view_t* views, void* stream);
/* Chain rule of the conversion above: grad_views (N,12: dR_p3d row-major, dT) -> grad_R_cv (N,3,3),
 * grad_t_cv (N,3), both overwritten. */
int32_t mr_view_grads_to_opencv(const float* grad_views, int64_t N, float* grad_R_cv, float* grad_t_cv, void* stream);

/* ---------------- mesh helpers ---------------- */
/* Meshes.verts_normals_packed: n_f = (v2-v1) x (v0-v1), summed in (corner, face) order, normalized (eps 1e-6).
 * vnormals_raw (V,3) keeps the unnormalized sums for the backward. */
int32_t mr_vertex_normals(const float* verts, int64_t V, const int32_t* faces, int64_t F, const int32_t* vadj_ptr,
                          const int32_t* vadj, float* vnormals, float* vnormals_raw, void* stream);

/* ---------------- fused render (one raster pass -> depth, silhouette, rgb) ---------------- */
size_t mr_render_workspace(int64_t N, int64_t F, int32_t H, int32_t W, int32_t max_faces_per_bin);
/* The same for N distinct meshes of F faces in total (mr_mesh_t.view_face_first set). */
size_t mr_render_workspace_meshes(int64_t N, int64_t F, int32_t H, int32_t W, int32_t max_faces_per_bin);
/* Outputs (each optional per out_flags): depth (N,H,W), silhouette (N,H,W), rgb (N,H,W,C);
 * pix_to_face32 (N,H,W) int32 packed face id n*F+f (distinct meshes: the union face id) or -1 — optional (NULL: not written; the
 * backward does not need it: the workspace keeps each non-empty 8x8 tile's winners and their fragments).
 * cam_centers (Nc,3) world-space specular camera centres, Nc in {1, N}. */
int32_t mr_render_forward(const mr_mesh_t* mesh, const mr_view_t* views, int64_t N, const float* cam_centers,
                          int64_t num_cam_centers, const mr_raster_settings_t* rs, const mr_shade_params_t* sp,
                          float* depth, float* silhouette, float* rgb, int32_t* pix_to_face32, void* workspace,
                          size_t workspace_bytes, void* stream);
/* OpenCV camera poses as DifferentiableRenderer takes them (torch_renderer.py:73-80): R_cv (N,3,3),
 * t_cv (N,3), intrinsics rows {ax, bx, ay, by} (N,4); *_stride = floats between consecutive views
 * (0 broadcasts one row). */
typedef struct mr_opencv_poses {
  const float* R;
  int64_t R_stride;
  const float* t;
  int64_t t_stride;
  const float* intr;
  int64_t intr_stride;
} mr_opencv_poses_t;
/* mr_render_forward for OpenCV poses: the pose conversion (mr_views_from_opencv) happens inside the
 * forward's first launch, which also writes the converted records to views_out (N) for the backward
 * (mr_render_backward_opencv). Replaces DifferentiableRenderer._camera_pose_from_opencv_to_pytorch +
 * the render call (torch_renderer.py:73-80, :110-121, :155-159). */
int32_t mr_render_forward_opencv(const mr_mesh_t* mesh, const mr_opencv_poses_t* poses, mr_view_t* views_out,
                                 int64_t N, const float* cam_centers, int64_t num_cam_centers,
                                 const mr_raster_settings_t* rs, const mr_shade_params_t* sp, float* depth,
                                 float* silhouette, float* rgb, int32_t* pix_to_face32, void* workspace,
                                 size_t workspace_bytes, void* stream);
/* mr_render_forward for PyTorch3D-convention poses given as strided device arrays (R (N,3,3), T (N,3),
 * intr (N,4); a batch stride of 0 broadcasts one row): the view records are packed by the forward's
 * first launch and written to views_out (N) for mr_render_backward — no host-side packing of R, T and
 * intr (upstream MeshRenderer(meshes, R=, T=) callers: camera_pose_optimizer.py:248-250,
 * mesh_deformer.py:197). */
int32_t mr_render_forward_poses(const mr_mesh_t* mesh, const mr_poses_t* poses, mr_view_t* views_out, int64_t N,
                                const float* cam_centers, int64_t num_cam_centers, const mr_raster_settings_t* rs,
                                const mr_shade_params_t* sp, float* depth, float* silhouette, float* rgb,
                                int32_t* pix_to_face32, void* workspace, size_t workspace_bytes, void* stream);
/* Backward from upstream grads (each may be NULL when not requested in out_flags).
 * Writes grad_verts (V,3), grad_views (N,12), grad_vcolors (V,3; tex_kind 1 only, may be NULL).
 * `fwd_workspace` must be the one passed to the matching mr_render_forward: its face records and
 * covered-pixel list are reused (nothing is re-rasterized). */
/* The caller's renderers often shade the SAME raster several times per step (camera_pose_optimizer.py:
 * 244,248,250: rasterizer zbuf, silhouette and Phong renders of identical meshes / R / T / cameras /
 * settings). mr_render_reshade shades again from a workspace a previous mr_render_forward[_opencv]
 * filled for the same mesh geometry, views (`views` = that call's view records), sizes and raster
 * settings: it skips projection, binning and rasterization (the winners, face records and fragments
 * are reused) and runs vertex normals (when needed) -> this call's shading records (out_flags slot,
 * MR_SREC_SLOT(k), k != the slots of the other calls still to be differentiated) -> background ->
 * covered pixels. Outputs bitwise those of a full mr_render_forward with the same arguments. Its
 * backward is mr_render_backward[_opencv] over the same workspace with the same out_flags slot. */
int32_t mr_render_reshade(const mr_mesh_t* mesh, const mr_view_t* views, int64_t N, const float* cam_centers,
                          int64_t n_cam_centers, const mr_raster_settings_t* s, const mr_shade_params_t* sp,
                          float* depth, float* sil, float* rgb, int32_t* pix_to_face, void* workspace,
                          size_t workspace_bytes, void* stream);

size_t mr_render_backward_workspace(int64_t N, int64_t V, int64_t F, int32_t H, int32_t W);
int32_t mr_render_backward(const mr_mesh_t* mesh, const float* vnormals_raw, const mr_view_t* views, int64_t N,
                           const float* cam_centers, int64_t num_cam_centers, const mr_raster_settings_t* rs,
                           const mr_shade_params_t* sp, const float* grad_depth,
                           const float* grad_silhouette, const float* grad_rgb, const void* fwd_workspace,
                           void* bwd_workspace, size_t bwd_workspace_bytes, float* grad_verts, float* grad_views,
                           float* grad_vcolors, void* stream);
/* Same as mr_render_backward for views built by mr_views_from_opencv: the per-view pose
 * gradients are written straight in the OpenCV frame, grad_R_cv (N,3,3) and grad_t_cv (N,3)
 * (the chain rule of mr_view_grads_to_opencv fused into the reduction; torch_renderer.py:73-80). */
int32_t mr_render_backward_opencv(const mr_mesh_t* mesh, const float* vnormals_raw, const mr_view_t* views, int64_t N,
                                  const float* cam_centers, int64_t num_cam_centers, const mr_raster_settings_t* rs,
                                  const mr_shade_params_t* sp, const float* grad_depth,
                                  const float* grad_silhouette, const float* grad_rgb, const void* fwd_workspace,
                                  void* bwd_workspace, size_t bwd_workspace_bytes, float* grad_verts,
                                  float* grad_R_cv, float* grad_t_cv, float* grad_vcolors, void* stream);

/* ---------------- soft shading over stored fragments (K >= 1) ---------------- */
/* SoftPhongShader (out_flags = MR_OUT_RGB: phong_shading + softmax_rgb_blend) or SoftSilhouetteShader
 * (MR_OUT_SIL: sigmoid_alpha_blend, rgb = 1) applied to the fragments of mr_rasterize_meshes
 * (pix_to_face (N,H,W,K) packed ids n*F + f of ONE mesh shared by the N views, zbuf, bary
 * (original-face barycentrics), dists). rgba (N,H,W,4) is written. The workspace holds per-face
 * shading records and must be passed unchanged to the backward. */
size_t mr_shade_fragments_workspace(int64_t F);
int32_t mr_shade_fragments_forward(const mr_mesh_t* mesh, const int64_t* pix_to_face, const float* zbuf,
                                   const float* bary, const float* dists, int64_t N, int32_t H, int32_t W, int32_t K,
                                   const float* cam_centers, int64_t num_cam_centers, const mr_shade_params_t* sp,
                                   float* rgba, void* workspace, size_t workspace_bytes, void* stream);
/* Backward from grad_rgba (N,H,W,4): grad_zbuf / grad_dists (N,H,W,K), grad_bary (N,H,W,K,3) (for
 * mr_rasterize_meshes_backward), grad_verts (V,3) of the attribute path (interpolated world positions and
 * vertex normals), grad_vcolors (V,3; tex_kind 1), grad_tex_rgba (Ht,Wt,4) and grad_verts_uvs
 * (num_verts_uvs,2) (tex_kind 2; either may be NULL). All are overwritten. Gradients that are zero by
 * construction may be NULL: grad_zbuf and grad_bary with MR_OUT_SIL (the silhouette blend reads only
 * the distances), grad_zbuf and grad_dists with MR_OUT_HARD (hard_rgb_blend reads neither). */
size_t mr_shade_fragments_backward_workspace(int64_t V, int64_t F);
int32_t mr_shade_fragments_backward(const mr_mesh_t* mesh, const float* vnormals_raw, const int64_t* pix_to_face,
                                    const float* zbuf, const float* bary, const float* dists, int64_t N, int32_t H,
                                    int32_t W, int32_t K, const float* cam_centers, int64_t num_cam_centers,
                                    const mr_shade_params_t* sp, const float* grad_rgba, const void* fwd_workspace,
                                    void* bwd_workspace, size_t bwd_workspace_bytes, float* grad_zbuf,
                                    float* grad_bary, float* grad_dists, float* grad_verts, float* grad_vcolors,
                                    float* grad_tex_rgba, float* grad_verts_uvs, int64_t num_verts_uvs,
                                    void* stream);

/* MeshRenderer(MeshRasterizer(faces_per_pixel = K, 2 <= K <= 64), SoftSilhouetteShader(sigma)) for ONE
 * mesh shared by N views (deform_mesh_with_color.py:153-165) in one pass: the K-deep fragments are blended
 * as they are produced and never written. rgba (N,H,W,4) must hold the background (1, 1, 1, 0) on entry
 * (tiles no face reaches are not written); it gets (1, 1, 1, 1 - prod_k (1 - sigmoid(-d_k / sigma))),
 * bitwise mr_rasterize_meshes_world + mr_shade_fragments_forward(MR_OUT_SIL). views_out / face_verts as
 * mr_rasterize_meshes_world. The workspace keeps each tile's fragments compactly for the backward, which
 * writes grad_face_verts (N*F,3,3) for mr_project_faces_backward: the chain of
 * mr_shade_fragments_backward(MR_OUT_SIL) and mr_rasterize_meshes_backward without fragment-gradient
 * tensors. MR_EUNSUPPORTED for grids the per-view binning does not take (the caller then runs the
 * two-step path). */
size_t mr_soft_silhouette_workspace(int64_t N, int64_t F, int32_t H, int32_t W, int32_t K, int32_t max_faces_per_bin);
int32_t mr_soft_silhouette_forward(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                   const mr_poses_t* poses, int64_t N, const mr_raster_settings_t* s, float sigma,
                                   mr_view_t* views_out, float* face_verts, float* rgba, void* workspace,
                                   size_t workspace_bytes, void* stream);
int32_t mr_soft_silhouette_backward(const float* face_verts, int64_t N, int64_t F, const mr_raster_settings_t* s,
                                    float sigma, const float* grad_rgba, const void* workspace, float* grad_face_verts,
                                    void* stream);

/* ---------------- instrumentation ---------------- */

/* camera_pose_optimizer.py:257-276 Model.calc_loss fused: sil_loss =
 * L1Loss(sil, mask), hloss = HuberLoss(delta)(depth[mask], depth_ref[mask]), color_loss =
 * MSELoss(rgb, rgb_ref); out[4] = {sil_loss + hloss + w_color * color_loss, sil_loss, hloss,
 * color_loss} (device). All inputs hold npix = N*H*W pixels; rgb may be an RGBA view
 * (rgb_stride 4); mask is a bool (uint8) tensor. Deterministic (fixed-order reductions). The
 * backward writes dL/d{depth, sil, rgb (npix,3)} given the device scalar dL/dtotal and the
 * forward's workspace. */
size_t mr_pose_loss_workspace(int64_t npix);
int32_t mr_pose_loss_forward(const float* depth, const float* sil, int64_t sil_stride, const float* rgb,
                             int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                             int64_t npix, float delta, float w_color, float* out, void* ws, size_t ws_bytes,
                             void* stream);
/* sil_stride 1: sil is (npix); 4: sil is channel 3 of an (npix, 4) RGBA tensor (the SoftSilhouetteShader
 * image the reference slices with [..., 3]), read in place. rgb_stride 3 or 4 likewise. The gradients
 * come back in the same layouts, for the whole tensors the views were taken from: g_sil (npix) or
 * (npix, 4) RGBA with zero RGB, g_rgb (npix, 3) or (npix, 4) with zero alpha — what the slices'
 * backward would produce, without its zero-filled buffer and strided copy. */
int32_t mr_pose_loss_backward(const float* depth, const float* sil, int64_t sil_stride, const float* rgb,
                              int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                              int64_t npix, float delta, float w_color, const float* g_total, const void* fwd_ws,
                              float* g_depth, float* g_sil, float* g_rgb, void* stream);
/* The forward that also writes the gradients for dL/dtotal = 1 (same layouts as mr_pose_loss_backward):
 * the loss is linear in dL/dtotal, so one pass over the inputs serves both directions;
 * mr_pose_loss_scale then multiplies the three buffers by the device scalar dL/dtotal in place (a no-op
 * grid when it is 1). total (1 float) and terms (3: sil_loss, hloss, color_loss) are separate outputs;
 * the gradient buffers are all three or all NULL (the loss alone); RGBA gradient buffers 16-B aligned. */
int32_t mr_pose_loss_forward_grad(const float* depth, const float* sil, int64_t sil_stride, const float* rgb,
                                  int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                                  int64_t npix, float delta, float w_color, float* total, float* terms, void* ws,
                                  size_t ws_bytes, float* g_depth, float* g_sil, float* g_rgb, void* stream);
int32_t mr_pose_loss_scale(const float* g_total, int64_t npix, int64_t sil_stride, int64_t rgb_stride, float* g_depth,
                           float* g_sil, float* g_rgb, void* stream);

/* upstream pytorch3d.transforms.quaternion_to_matrix (camera_pose_optimizer.py:241: the 7-vector
 * pose's real-first quaternion, not renormalised: two_s = 2 / |q|^2) for N quaternions q (rows
 * q_stride floats apart) -> R (N,3,3), torch's operation order (bitwise the elementwise torch
 * formula); the backward writes dL/dq (N,4) from dL/dR. One launch each instead of ~90 tiny torch
 * kernels per optimiser step. */
int32_t mr_quaternion_to_matrix(const float* q, int64_t q_stride, int64_t N, float* R, void* stream);
int32_t mr_quaternion_to_matrix_backward(const float* q, int64_t q_stride, const float* grad_R, int64_t N,
                                         float* grad_q, void* stream);

/* Work counters left in `workspace` by the last mr_render_forward / mr_rasterize_meshes that used it
 * (same N, total faces, H, W, max_faces_per_bin). Synchronises `stream`; for benchmarks and tools.
 * out[0] = (tile, face) list entries, out[1] = raster work units, out[2] = non-empty 8x8 tiles,
 * out[3] = covered pixels. */
/* 1 when a batch of N views with total_faces face instances at H x W takes the per-view binning
 * (k_bin_rect_* -> k_bin_view: tile grids of <= 16,384 8x8 tiles, <= 256 a side), 0 when it takes
 * count -> scan -> fill. The fused soft silhouette and the deterministic face gradients need the former. */
int32_t mr_per_view_binning(int64_t N, int64_t total_faces, int32_t H, int32_t W);

int32_t mr_workspace_stats(const void* workspace, int64_t N, int64_t total_faces, int32_t H, int32_t W,
                           int32_t max_faces_per_bin, int64_t* out, void* stream);

/* The 8 raw work counters at the head of a forward workspace (same sizes as the forward that used
 * it): [0] work units, [1] non-empty tiles, [3] kept soft-silhouette fragments, [4..5] list entries
 * (u64), [6] tiles the K-deep raster walked near-to-far (its depth-ordered list walk). Synchronises
 * `stream`; for tests and tools. */
int32_t mr_workspace_counters(const void* workspace, int64_t N, int64_t total_faces, int32_t H, int32_t W,
                              int32_t max_faces_per_bin, int32_t* out8, void* stream);

/* Per-kernel timing with HIP events recorded on each launch's stream (bench.py).
 * enable=1 clears and starts collection; mr_timing_read synchronizes on the
 * recorded events and returns, per kernel id, launches and summed ms. */
int32_t mr_timing_enable(int32_t enable);
int32_t mr_timing_read(int32_t* launches, double* total_ms, int32_t n);
const char* mr_timing_kernel_name(int32_t k);
int32_t mr_timing_kernel_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MI355R_H */
