// mi355r — torch glue in C++: the autograd nodes of the fused render, the pose loss and quaternion_to_matrix.
//
// The reference callers run the render eagerly, several times per optimiser step (camera_pose_optimizer.py:
// 244-250: three renders of one pose batch; mesh_deformer.py:197: five single-view renders), so the host work
// around each native call is on the step's critical path. This node does, for one call, what the Python
// autograd.Function did — allocate the outputs and the workspace, fill mr_mesh_t / mr_poses_t, call
// mr_render_forward_poses / _opencv / mr_render_reshade, and in the backward mr_render_backward[_opencv] —
// without Python on either side: the backward runs inside autograd's device thread with no GIL round trip.
// Everything arithmetic stays behind the C ABI (include/mi355r.h); this file only marshals tensors.
// Built by torch_renderer_amd/_build.py against torch's headers. It does not link libmi355r.so: _lib.py
// hands it the addresses of the C ABI functions of the library it loaded (init()), so the node always calls
// the same library as the rest of the package (MI355R_LIB experiment builds included).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

#include "mi355r.h"

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

namespace {

// The C ABI entry points this node calls, from the library _lib.py loaded.
struct Abi {
  decltype(&mr_last_error) last_error = nullptr;
  decltype(&mr_render_workspace) workspace = nullptr;
  decltype(&mr_render_workspace_meshes) workspace_meshes = nullptr;
  decltype(&mr_render_reshade) reshade = nullptr;
  decltype(&mr_render_forward_opencv) forward_opencv = nullptr;
  decltype(&mr_render_forward_poses) forward_poses = nullptr;
  decltype(&mr_render_backward_workspace) backward_workspace = nullptr;
  decltype(&mr_render_backward) backward = nullptr;
  decltype(&mr_render_backward_opencv) backward_opencv = nullptr;
  decltype(&mr_pose_loss_workspace) loss_workspace = nullptr;
  decltype(&mr_pose_loss_forward_grad) loss_forward_grad = nullptr;
  decltype(&mr_pose_loss_scale) loss_scale = nullptr;
  decltype(&mr_pose_loss_backward) loss_backward = nullptr;
  decltype(&mr_quaternion_to_matrix) quat = nullptr;
  decltype(&mr_quaternion_to_matrix_backward) quat_backward = nullptr;
} g_abi;

// The torch current stream of t's device (the autograd engine sets the forward's stream for the backward).
hipStream_t stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check(int32_t rc) {
  if (rc == MR_OK) return;
  const char* e = g_abi.last_error();
  TORCH_CHECK_NOT_IMPLEMENTED(rc != MR_EUNSUPPORTED, "mi355r: ", e);  // Python: NotImplementedError
  TORCH_CHECK(false, "mi355r error ", rc, ": ", e);
}

template <typename T>
T* dptr(const Tensor& t) {
  return t.defined() ? (T*)t.data_ptr() : nullptr;
}

// A float tensor whose per-view rows are contiguous (elements between views in `stride`; 0 broadcasts
// one row), as kernels.py _batch_stride.
Tensor batch_rows(Tensor t, int64_t row, int64_t& stride) {
  t = t.reshape({-1, row});
  if (t.scalar_type() != at::kFloat) t = t.to(at::kFloat);
  if (t.stride(1) != 1) t = t.contiguous();
  stride = t.size(0) > 1 ? t.stride(0) : 0;
  return t;
}

Tensor f32c(const Tensor& t) {
  Tensor x = t.scalar_type() == at::kFloat ? t : t.to(at::kFloat);
  return x.is_contiguous() ? x : x.contiguous();
}

// Whether a backward already consumed a forward workspace's face-gradient totals (the forward clears them;
// the first backward over it may skip the clear: MR_GRAD_ROWS_CLEARED). Keyed by the workspace's address:
// a fresh forward resets its entry; an address the map does not know is treated as used (a clear).
std::mutex g_used_mu;
std::unordered_map<const void*, bool> g_used;
void ws_reset(const void* p) {
  std::lock_guard<std::mutex> l(g_used_mu);
  if (g_used.size() > 4096) g_used.clear();
  g_used[p] = false;
}
bool ws_first_use(const void* p) {
  std::lock_guard<std::mutex> l(g_used_mu);
  auto it = g_used.find(p);
  if (it == g_used.end() || it->second) return false;
  it->second = true;
  return true;
}

// Non-differentiable arguments of one call (a struct, so autograd's argument walk does not take them
// as inputs).
struct RenderArgs {
  Tensor faces, vptr, vadj, intr, cc;
  Tensor verts_uvs, faces_uvs, tex_rgba, tex_u8, tex_lut;
  int64_t tex_kind = 0;
  Tensor ffirst, fcount;  // distinct meshes (undefined: one shared mesh)
  int64_t fmax = 0;
  std::string rs, sp;     // mr_raster_settings_t, mr_shade_params_t (out_flags as the call wants them)
  int64_t flags = 0;      // bit 0: OpenCV poses; bit 1: pix_to_face32 output
  Tensor ws, views;       // reshade: the shared raster's workspace and view records (undefined: a forward)
  int64_t slot = 0;       // ShadeRec slot of a reshade (mr_render_reshade)
};

mr_mesh_t make_mesh(const Tensor& v, const Tensor& vcol, const RenderArgs& a, const Tensor& vn) {
  mr_mesh_t m;
  std::memset(&m, 0, sizeof(m));
  m.verts = dptr<float>(v);
  m.V = v.size(0);
  m.faces = dptr<int32_t>(a.faces);
  m.F = a.faces.size(0);
  m.vadj_ptr = dptr<int32_t>(a.vptr);
  m.vadj = dptr<int32_t>(a.vadj);
  m.vnormals = dptr<float>(vn);
  m.tex_kind = (int32_t)a.tex_kind;
  m.vcolors = dptr<float>(vcol);
  m.verts_uvs = dptr<float>(a.verts_uvs);
  m.faces_uvs = dptr<int32_t>(a.faces_uvs);
  m.tex_rgba = dptr<float>(a.tex_rgba);
  if (a.tex_rgba.defined()) {
    m.tex_h = (int32_t)a.tex_rgba.size(0);
    m.tex_w = (int32_t)a.tex_rgba.size(1);
  }
  if (a.tex_u8.defined() && a.tex_lut.defined()) {
    m.tex_u8 = dptr<uint8_t>(a.tex_u8);
    m.tex_lut = dptr<float>(a.tex_lut);
  }
  if (a.ffirst.defined()) {
    m.view_face_first = dptr<int64_t>(a.ffirst);
    m.view_face_count = dptr<int64_t>(a.fcount);
    m.max_view_faces = a.fmax;
  }
  return m;
}

struct RenderViewsFn : public torch::autograd::Function<RenderViewsFn> {
  // outputs: [depth] [sil] [rgb] [p2f32] ws views (as the shade params' out_flags ask)
  static variable_list forward(AutogradContext* ctx, Tensor verts, Tensor R, Tensor T, Tensor vcolors,
                               RenderArgs a) {
    ctx->set_materialize_grads(false);
    mr_raster_settings_t rs;
    mr_shade_params_t sp;
    TORCH_CHECK(a.rs.size() == sizeof(rs) && a.sp.size() == sizeof(sp), "mi355r: settings blob sizes");
    std::memcpy(&rs, a.rs.data(), sizeof(rs));
    std::memcpy(&sp, a.sp.data(), sizeof(sp));
    const bool pose_cv = (a.flags & 1) != 0, want_p2f = (a.flags & 2) != 0, reuse = a.ws.defined();
    const auto dev = verts.device();
    Tensor v = f32c(verts.detach());
    const bool has_vcol = vcolors.numel() > 0;  // (an empty placeholder when the mesh has no vertex colours)
    Tensor vcol = has_vcol ? f32c(vcolors.detach()) : Tensor();
    Tensor cc = f32c(a.cc).reshape({-1, 3});
    const int64_t Rn = R.numel() / 9, Tn = T.numel() / 3, In = a.intr.numel() / 4;
    const int64_t N = reuse ? a.views.size(0) : std::max(Rn, std::max(Tn, In));
    const int64_t H = rs.H, W = rs.W;
    auto fo = at::TensorOptions().dtype(at::kFloat).device(dev);
    Tensor vn, raw;
    if (sp.light_kind == 0) {  // computed by the forward's first launch (mesh.vnormals_out)
      vn = at::empty_like(v);
      raw = at::empty_like(v);
    }
    mr_mesh_t m = make_mesh(v, vcol, a, vn);
    if (vn.defined()) {
      m.vnormals_out = dptr<float>(vn);
      m.vraw_out = dptr<float>(raw);
    }
    const int of = sp.out_flags;
    Tensor depth, sil, rgb, p2f;
    if (of & MR_OUT_DEPTH) depth = at::empty({N, H, W}, fo);
    if (of & MR_OUT_SIL) sil = (of & MR_OUT_SIL_RGBA) ? at::empty({N, H, W, 4}, fo) : at::empty({N, H, W}, fo);
    if (of & MR_OUT_RGB) rgb = at::empty({N, H, W, (int64_t)sp.rgb_channels}, fo);
    if (want_p2f) p2f = at::empty({N, H, W}, at::TensorOptions().dtype(at::kInt).device(dev));
    Tensor ws = a.ws, views = a.views;
    const int64_t Fn = a.faces.size(0);
    const size_t wsb = a.ffirst.defined() ? g_abi.workspace_meshes(N, Fn, (int32_t)H, (int32_t)W, rs.max_faces_per_bin)
                                          : g_abi.workspace(N, Fn, (int32_t)H, (int32_t)W, rs.max_faces_per_bin);
    const hipStream_t st = stream_of(v);
    if (reuse) {
      TORCH_CHECK(ws.numel() >= (int64_t)wsb, "mi355r: reshade workspace too small");
      sp.out_flags |= (int32_t)(a.slot << MR_SREC_SLOT_SHIFT);
      check(g_abi.reshade(&m, (const mr_view_t*)views.data_ptr(), N, dptr<float>(cc), cc.size(0), &rs, &sp,
                              dptr<float>(depth), dptr<float>(sil), dptr<float>(rgb), dptr<int32_t>(p2f), ws.data_ptr(),
                              wsb, st));
    } else {
      ws = at::empty({(int64_t)wsb}, at::TensorOptions().dtype(at::kByte).device(dev));
      views = at::empty({N, 16}, fo);
      int64_t sR, sT, sI;
      Tensor Rb = batch_rows(R.detach(), 9, sR), Tb = batch_rows(T.detach(), 3, sT), Ib = batch_rows(a.intr, 4, sI);
      ws_reset(ws.data_ptr());
      if (pose_cv) {
        mr_opencv_poses_t p{dptr<float>(Rb), sR, dptr<float>(Tb), sT, dptr<float>(Ib), sI};
        check(g_abi.forward_opencv(&m, &p, (mr_view_t*)views.data_ptr(), N, dptr<float>(cc), cc.size(0), &rs, &sp,
                                       dptr<float>(depth), dptr<float>(sil), dptr<float>(rgb), dptr<int32_t>(p2f),
                                       ws.data_ptr(), wsb, st));
      } else {
        mr_poses_t p{dptr<float>(Rb), sR, dptr<float>(Tb), sT, dptr<float>(Ib), sI};
        check(g_abi.forward_poses(&m, &p, (mr_view_t*)views.data_ptr(), N, dptr<float>(cc), cc.size(0), &rs, &sp,
                                      dptr<float>(depth), dptr<float>(sil), dptr<float>(rgb), dptr<int32_t>(p2f),
                                      ws.data_ptr(), wsb, st));
      }
    }
    // saved for the backward: every tensor the mesh struct points into, the view records, the workspace
    ctx->save_for_backward({v, vcol, views, cc, ws, vn, raw, a.faces, a.vptr, a.vadj, a.verts_uvs, a.faces_uvs,
                            a.tex_rgba, a.tex_u8, a.tex_lut, a.ffirst, a.fcount});
    ctx->saved_data["rs"] = std::string((const char*)&rs, sizeof(rs));
    ctx->saved_data["sp"] = std::string((const char*)&sp, sizeof(sp));  // (its slot bits included)
    ctx->saved_data["tex_kind"] = a.tex_kind;
    ctx->saved_data["fmax"] = a.fmax;
    ctx->saved_data["pose_cv"] = pose_cv;
    ctx->saved_data["vcol"] = has_vcol;
    variable_list outs;
    for (const Tensor* t : {&depth, &sil, &rgb})
      if (t->defined()) outs.push_back(*t);
    if (p2f.defined()) {
      ctx->mark_non_differentiable({p2f});
      outs.push_back(p2f);
    }
    ctx->mark_non_differentiable({ws, views});
    outs.push_back(ws);
    outs.push_back(views);
    return outs;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto s = ctx->get_saved_variables();
    const Tensor &v = s[0], &vcol = s[1], &views = s[2], &cc = s[3], &ws = s[4], &vn = s[5], &raw = s[6];
    RenderArgs a;
    a.faces = s[7]; a.vptr = s[8]; a.vadj = s[9];
    a.verts_uvs = s[10]; a.faces_uvs = s[11]; a.tex_rgba = s[12]; a.tex_u8 = s[13]; a.tex_lut = s[14];
    a.ffirst = s[15]; a.fcount = s[16];
    a.tex_kind = ctx->saved_data["tex_kind"].toInt();
    a.fmax = ctx->saved_data["fmax"].toInt();
    const bool pose_cv = ctx->saved_data["pose_cv"].toBool(), has_vcol = ctx->saved_data["vcol"].toBool();
    mr_raster_settings_t rs;
    mr_shade_params_t sp;
    const std::string rsb = ctx->saved_data["rs"].toStringRef(), spb = ctx->saved_data["sp"].toStringRef();
    std::memcpy(&rs, rsb.data(), sizeof(rs));
    std::memcpy(&sp, spb.data(), sizeof(sp));
    // the image gradients that arrived (absent ones: NULL, no zero tensors), in the outputs' order
    Tensor gD, gS, gC;
    size_t gi = 0;
    if (sp.out_flags & MR_OUT_DEPTH) gD = grads[gi++];
    if (sp.out_flags & MR_OUT_SIL) gS = grads[gi++];
    if (sp.out_flags & MR_OUT_RGB) gC = grads[gi++];
    sp.out_flags &= ~((gD.defined() ? 0 : (MR_OUT_DEPTH | MR_OUT_ZBUF)) | (gS.defined() ? 0 : (MR_OUT_SIL | MR_OUT_SIL_RGBA)) |
                      (gC.defined() ? 0 : MR_OUT_RGB));
    if (ws_first_use(ws.data_ptr())) sp.out_flags |= MR_GRAD_ROWS_CLEARED;  // the forward cleared the face totals
    if (gD.defined()) gD = f32c(gD);
    if (gS.defined()) gS = f32c(gS);
    if (gC.defined()) gC = f32c(gC);
    mr_mesh_t m = make_mesh(v, vcol, a, vn);
    const int64_t N = views.size(0);
    auto fo = at::TensorOptions().dtype(at::kFloat).device(v.device());
    Tensor gverts = at::empty_like(v), gcol = has_vcol ? at::empty_like(v) : Tensor();
    const size_t bwb = g_abi.backward_workspace(N, v.size(0), a.faces.size(0), rs.H, rs.W);
    Tensor bws = at::empty({(int64_t)bwb}, at::TensorOptions().dtype(at::kByte).device(v.device()));
    const hipStream_t st = stream_of(v);
    Tensor gR, gT;
    if (pose_cv) {  // pose grads straight in the OpenCV frame
      gR = at::empty({N, 3, 3}, fo);
      gT = at::empty({N, 3}, fo);
      check(g_abi.backward_opencv(&m, dptr<float>(raw), (const mr_view_t*)views.data_ptr(), N, dptr<float>(cc),
                                      cc.size(0), &rs, &sp, dptr<float>(gD), dptr<float>(gS), dptr<float>(gC),
                                      ws.data_ptr(), bws.data_ptr(), bwb, dptr<float>(gverts), dptr<float>(gR),
                                      dptr<float>(gT), dptr<float>(gcol), st));
    } else {
      Tensor gviews = at::empty({N, 12}, fo);
      check(g_abi.backward(&m, dptr<float>(raw), (const mr_view_t*)views.data_ptr(), N, dptr<float>(cc), cc.size(0),
                               &rs, &sp, dptr<float>(gD), dptr<float>(gS), dptr<float>(gC), ws.data_ptr(),
                               bws.data_ptr(), bwb, dptr<float>(gverts), dptr<float>(gviews), dptr<float>(gcol), st));
      gR = gviews.narrow(1, 0, 9).reshape({N, 3, 3});
      gT = gviews.narrow(1, 9, 3);
    }
    return {gverts, gR, gT, gcol, Tensor()};  // (none for the RenderArgs argument)
  }
};

// kernels.render_views' native call. Returns [depth] [sil] [rgb] [p2f32] ws views.
variable_list render_views(Tensor verts, Tensor R, Tensor T, c10::optional<Tensor> vcolors, Tensor faces, Tensor vptr,
                           Tensor vadj, Tensor intr, Tensor cc, int64_t tex_kind, c10::optional<Tensor> verts_uvs,
                           c10::optional<Tensor> faces_uvs, c10::optional<Tensor> tex_rgba, c10::optional<Tensor> tex_u8,
                           c10::optional<Tensor> tex_lut, c10::optional<Tensor> ffirst, c10::optional<Tensor> fcount,
                           int64_t fmax, std::string rs, std::string sp, int64_t flags, c10::optional<Tensor> ws,
                           c10::optional<Tensor> views, int64_t slot) {
  TORCH_CHECK(g_abi.forward_poses != nullptr, "mi355r: _mr_torch.init() was not called");
  TORCH_CHECK(verts.is_cuda() && R.is_cuda() && T.is_cuda() && faces.is_cuda(),
              "mi355r renders HIP tensors only (no CPU fallback): move the mesh and cameras to the GPU");
  RenderArgs a;
  a.faces = faces; a.vptr = vptr; a.vadj = vadj; a.intr = intr; a.cc = cc;
  a.tex_kind = tex_kind;
  a.verts_uvs = verts_uvs.value_or(Tensor()); a.faces_uvs = faces_uvs.value_or(Tensor());
  a.tex_rgba = tex_rgba.value_or(Tensor()); a.tex_u8 = tex_u8.value_or(Tensor()); a.tex_lut = tex_lut.value_or(Tensor());
  a.ffirst = ffirst.value_or(Tensor()); a.fcount = fcount.value_or(Tensor()); a.fmax = fmax;
  a.rs = std::move(rs); a.sp = std::move(sp); a.flags = flags;
  a.ws = ws.value_or(Tensor()); a.views = views.value_or(Tensor()); a.slot = slot;
  // an absent vcolors travels as an empty tensor (autograd inputs must be defined tensors)
  Tensor vc = vcolors.has_value() && vcolors->defined() ? *vcolors : at::empty({0}, verts.options());
  return RenderViewsFn::apply(verts, R, T, vc, std::move(a));
}

// camera_pose_optimizer.py:257-276 calc_loss (losses.pose_loss): the forward writes the gradients for
// dL/dtotal = 1 with the loss (one pass); the first backward rescales them in place (mr_pose_loss_scale),
// a later one (retain_graph) recomputes them (mr_pose_loss_backward). sil / color may be the RGBA images
// whose [..., 3] / [..., :3] slices the caller passed (read in place, gradients in the RGBA layout).
struct LossArgs {
  Tensor mask, depth_ref, rgb_ref;
  double delta = 0.05, w_color = 0.01;
  bool sil_rgba = false, col_rgba = false;
  bool grads = false;  // a backward can follow (grad mode on and an image requires grad)
};

struct PoseLossFn : public torch::autograd::Function<PoseLossFn> {
  static variable_list forward(AutogradContext* ctx, Tensor depth, Tensor sil_in, Tensor color_in, LossArgs a) {
    const int64_t npix = depth.numel();
    const int64_t s_stride = a.sil_rgba ? 4 : 1, c_stride = a.col_rgba ? 4 : 3;
    TORCH_CHECK(a.rgb_ref.size(-1) == 3 && color_in.size(-1) == c_stride, "color and rgb_ref must end in 3 channels");
    TORCH_CHECK(sil_in.numel() == s_stride * npix && a.mask.numel() == npix && a.depth_ref.numel() == npix &&
                    color_in.numel() == c_stride * npix && a.rgb_ref.numel() == 3 * npix,
                "pose_loss: inputs must have one element per pixel (per channel) of depth (no broadcasting)");
    const auto dev = depth.device();
    Tensor d = f32c(depth.detach());
    Tensor sl = a.sil_rgba ? sil_in.detach() : f32c(sil_in.detach());
    Tensor c = a.col_rgba ? color_in.detach() : f32c(color_in.detach());
    Tensor m = a.mask.detach().to(at::kBool).contiguous().view(at::kByte);
    Tensor dr = f32c(a.depth_ref.detach()), rr = f32c(a.rgb_ref.detach());
    auto fo = at::TensorOptions().dtype(at::kFloat).device(dev);
    const size_t wsb = g_abi.loss_workspace(npix);
    Tensor ws = at::empty({(int64_t)wsb}, at::TensorOptions().dtype(at::kByte).device(dev));
    Tensor total = at::empty({}, fo), terms = at::empty({3}, fo);
    Tensor gd, gs, gc;
    const bool grads = a.grads;
    if (grads) {
      gd = at::empty_like(d);
      gs = at::empty({npix, s_stride}, fo);
      gc = at::empty({npix, c_stride}, fo);
    }
    const float* sp = dptr<float>(sl) + (a.sil_rgba ? 3 : 0);
    check(g_abi.loss_forward_grad(dptr<float>(d), sp, s_stride, dptr<float>(c), c_stride, dptr<uint8_t>(m),
                                  dptr<float>(dr), dptr<float>(rr), npix, (float)a.delta, (float)a.w_color,
                                  dptr<float>(total), dptr<float>(terms), ws.data_ptr(), wsb, dptr<float>(gd),
                                  dptr<float>(gs), dptr<float>(gc), stream_of(d)));
    ctx->save_for_backward({d, sl, c, m, dr, rr, ws, gd, gs, gc});
    ctx->saved_data["pre"] = grads;  // the forward's gradients are still unused
    ctx->saved_data["s_stride"] = s_stride;
    ctx->saved_data["c_stride"] = c_stride;
    ctx->saved_data["delta"] = a.delta;
    ctx->saved_data["w_color"] = a.w_color;
    ctx->saved_data["sh_d"] = depth.sizes().vec();
    ctx->saved_data["sh_s"] = sil_in.sizes().vec();
    ctx->saved_data["sh_c"] = color_in.sizes().vec();
    ctx->mark_non_differentiable({terms});
    return {total, terms};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    const Tensor &d = sv[0], &sl = sv[1], &c = sv[2], &m = sv[3], &dr = sv[4], &rr = sv[5], &ws = sv[6];
    const int64_t s_stride = ctx->saved_data["s_stride"].toInt(), c_stride = ctx->saved_data["c_stride"].toInt();
    const int64_t npix = d.numel();
    Tensor g = grads[0].defined() ? f32c(grads[0]).reshape({1}) : at::zeros({1}, d.options());
    const hipStream_t st = stream_of(d);
    Tensor gd, gs, gc;
    if (ctx->saved_data["pre"].toBool()) {  // the forward's gradients, scaled by dL/dtotal (first backward)
      ctx->saved_data["pre"] = false;
      gd = sv[7];
      gs = sv[8];
      gc = sv[9];
      check(g_abi.loss_scale(dptr<float>(g), npix, s_stride, c_stride, dptr<float>(gd), dptr<float>(gs),
                             dptr<float>(gc), st));
    } else {
      auto fo = d.options();
      gd = at::empty_like(d);
      gs = at::empty({npix, s_stride}, fo);
      gc = at::empty({npix, c_stride}, fo);
      const float* sp = dptr<float>(sl) + (s_stride == 4 ? 3 : 0);
      check(g_abi.loss_backward(dptr<float>(d), sp, s_stride, dptr<float>(c), c_stride, dptr<uint8_t>(m),
                                dptr<float>(dr), dptr<float>(rr), npix, (float)ctx->saved_data["delta"].toDouble(),
                                (float)ctx->saved_data["w_color"].toDouble(), dptr<float>(g), ws.data_ptr(),
                                dptr<float>(gd), dptr<float>(gs), dptr<float>(gc), st));
    }
    return {gd.reshape(ctx->saved_data["sh_d"].toIntVector()), gs.reshape(ctx->saved_data["sh_s"].toIntVector()),
            gc.reshape(ctx->saved_data["sh_c"].toIntVector()), Tensor()};
  }
};

// quaternion_to_matrix (camera_pose_optimizer.py:241) of real-part-first quaternions q (..., 4): one launch
// each way; q may be a strided slice (the pose's q[:, 3:], rows 7 floats apart).
struct QuatFn : public torch::autograd::Function<QuatFn> {
  static Tensor forward(AutogradContext* ctx, Tensor q) {
    Tensor q2 = q.detach();
    if (q2.scalar_type() != at::kFloat) q2 = q2.to(at::kFloat);
    q2 = q2.reshape({-1, 4});
    if (q2.stride(1) != 1 || (q2.size(0) > 1 && q2.stride(0) < 4)) q2 = q2.contiguous();
    const int64_t n = q2.size(0);
    Tensor out = at::empty({n, 3, 3}, q2.options());
    check(g_abi.quat(dptr<float>(q2), q2.stride(0), n, dptr<float>(out), stream_of(q2)));
    ctx->save_for_backward({q2});
    ctx->saved_data["shape"] = q.sizes().vec();
    auto os = q.sizes().vec();
    os.back() = 3;
    os.push_back(3);
    return out.reshape(os);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const Tensor q2 = ctx->get_saved_variables()[0];
    const int64_t n = q2.size(0);
    Tensor gR = f32c(grads[0]);
    Tensor gq = at::empty({n, 4}, q2.options());
    check(g_abi.quat_backward(dptr<float>(q2), q2.stride(0), dptr<float>(gR), n, dptr<float>(gq), stream_of(q2)));
    return {gq.reshape(ctx->saved_data["shape"].toIntVector())};
  }
};

variable_list pose_loss(Tensor depth, Tensor sil, Tensor color, Tensor mask, Tensor depth_ref, Tensor rgb_ref,
                        double delta, double w_color, bool sil_rgba, bool col_rgba) {
  TORCH_CHECK(g_abi.loss_forward_grad != nullptr, "mi355r: _mr_torch.init() was not called");
  for (const Tensor* t : {&depth, &sil, &color, &mask, &depth_ref, &rgb_ref})
    TORCH_CHECK(t->is_cuda(), "mi355r: the MI355X path needs HIP device tensors (no CPU fallback)");
  LossArgs a;
  a.mask = mask; a.depth_ref = depth_ref; a.rgb_ref = rgb_ref;
  a.delta = delta; a.w_color = w_color; a.sil_rgba = sil_rgba; a.col_rgba = col_rgba;
  // (decided here: with no input requiring grad the node has no edges to ask)
  a.grads = at::GradMode::is_enabled() && (depth.requires_grad() || sil.requires_grad() || color.requires_grad());
  return PoseLossFn::apply(depth, sil, color, std::move(a));
}

Tensor quaternion_to_matrix(Tensor q) {
  TORCH_CHECK(g_abi.quat != nullptr, "mi355r: _mr_torch.init() was not called");
  return QuatFn::apply(q);
}

void init(const std::unordered_map<std::string, int64_t>& fn) {
  auto get = [&](const char* name) {
    auto it = fn.find(name);
    TORCH_CHECK(it != fn.end() && it->second != 0, "mi355r: C ABI function ", name, " missing");
    return (void*)it->second;
  };
  g_abi.last_error = (decltype(g_abi.last_error))get("mr_last_error");
  g_abi.workspace = (decltype(g_abi.workspace))get("mr_render_workspace");
  g_abi.workspace_meshes = (decltype(g_abi.workspace_meshes))get("mr_render_workspace_meshes");
  g_abi.reshade = (decltype(g_abi.reshade))get("mr_render_reshade");
  g_abi.forward_opencv = (decltype(g_abi.forward_opencv))get("mr_render_forward_opencv");
  g_abi.forward_poses = (decltype(g_abi.forward_poses))get("mr_render_forward_poses");
  g_abi.backward_workspace = (decltype(g_abi.backward_workspace))get("mr_render_backward_workspace");
  g_abi.backward = (decltype(g_abi.backward))get("mr_render_backward");
  g_abi.backward_opencv = (decltype(g_abi.backward_opencv))get("mr_render_backward_opencv");
  g_abi.loss_workspace = (decltype(g_abi.loss_workspace))get("mr_pose_loss_workspace");
  g_abi.loss_forward_grad = (decltype(g_abi.loss_forward_grad))get("mr_pose_loss_forward_grad");
  g_abi.loss_scale = (decltype(g_abi.loss_scale))get("mr_pose_loss_scale");
  g_abi.loss_backward = (decltype(g_abi.loss_backward))get("mr_pose_loss_backward");
  g_abi.quat = (decltype(g_abi.quat))get("mr_quaternion_to_matrix");
  g_abi.quat_backward = (decltype(g_abi.quat_backward))get("mr_quaternion_to_matrix_backward");
}

}  // namespace

#ifndef MR_TORCH_VERSION
#define MR_TORCH_VERSION "unknown"
#endif

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "mi355r torch glue: the fused render's autograd node (kernels.render_views)";
  // the torch this file was compiled against (_build.py passes torch.__version__): _lib.torch_ext() refuses a
  // stale build instead of failing later on a missing symbol or a mismatched ABI
  m.attr("built_with_torch") = MR_TORCH_VERSION;
  m.attr("built_with_cxx11_abi") = (bool)_GLIBCXX_USE_CXX11_ABI;
  m.def("init", &init, "the C ABI entry points (name -> address) of the loaded libmi355r.so");
  m.def("render_views", &render_views, "fused render forward (+ autograd backward) through the C ABI");
  m.def("pose_loss", &pose_loss, "calc_loss with its gradients (+ autograd backward) through the C ABI");
  m.def("quaternion_to_matrix", &quaternion_to_matrix, "quaternion_to_matrix (+ autograd backward)");
}
