// libtmdnet_torch.so -- the PyTorch dispatcher boundary of the HIP hot path.
//
// TorchScript and C++ (libtorch) consumers reach the kernels through registered operators, as they
// reach the reference's through its native op (reference torchmdnet/neighbors/neighbors.cpp:3-5,
// neighbors_cuda.cu:25-89):
//
//   torchmdnet_neighbors::get_neighbor_pairs   the reference schema, CUDA (= HIP) + AutogradCUDA;
//                                              a CPU kernel that raises (no CPU fallback).
//   tmdnet::neighbor_graph                     symmetric CSR list (row_ptr/src/dst/transpose) with
//                                              differentiable deltas/distances (OptimizedDistance,
//                                              reference models/utils.py:207-269)
//   tmdnet::edge_geometry                      RBF + CosineCutoff + unit vectors (utils.py:298-390,
//                                              torchmd_et.py:173-174)
//   tmdnet::nbr_embed                          NeighborEmbedding aggregation (utils.py:73-108)
//   tmdnet::et_message                         EquivariantMultiHeadAttention message + aggregate
//                                              (torchmd_et.py:314-347)
//   tmdnet::tn_embed / tmdnet::tn_message      TensorNet embedding aggregation / tensor message
//                                              passing (tensornet.py:295-332)
//
// Every op is a C++ autograd Function whose backward is another Function over the C ABI
// (include/tmdnet.h, libtmdnet_hip.so), so forces (create_graph=True, reference model.py:286-298)
// can be differentiated again for force-matching training: the neighbour geometry, the ET message
// and their backwards are HIP kernels to second order; the third order (and the second order of the
// edge geometry / neighbour embedding) differentiates a restatement in ATen ops.
//
// Host code only (compiled by g++ against the torch headers); no torch types cross the C ABI.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/autograd.h>
#include <torch/library.h>

#include <cmath>
#include <string>

#include "tmdnet.h"

namespace tmdt {

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::Function;
using torch::autograd::variable_list;

// ----------------------------------------------------------------------------- helpers
const char* status_name(int rc) {
  switch (rc) {
    case TMDNET_BAD_ARGUMENT: return "bad argument";
    case TMDNET_UNSUPPORTED: return "unsupported configuration";
    case TMDNET_LAUNCH_FAILED: return "kernel launch failed";
    case TMDNET_WORKSPACE_TOO_SMALL: return "workspace too small";
    default: return "error";
  }
}

void check(int rc, const char* what) {
  TORCH_CHECK(rc == TMDNET_OK, "torchmd-net_amd: ", what, " failed: ", status_name(rc));
}

void* stream_of(const Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int dcode(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return TMDNET_F32;
  if (t.scalar_type() == at::kDouble) return TMDNET_F64;
  TORCH_CHECK(false, "torchmd-net_amd: unsupported floating type ", t.scalar_type(), " (float32/float64)");
}

template <class P = void>
P* ptr(const Tensor& t) {
  return t.defined() ? static_cast<P*>(t.data_ptr()) : nullptr;
}

int ld(const Tensor& t) { return t.defined() ? static_cast<int>(t.stride(0)) : 0; }

// rows may be strided (views into fused projections); elements must be contiguous
Tensor rowmajor(const Tensor& t) { return (!t.defined() || t.stride(-1) == 1) ? t : t.contiguous(); }
Tensor contig(const Tensor& t) { return t.defined() ? t.contiguous() : t; }

void require_gpu(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), "torchmd-net_amd: ", what, " runs only on a ROCm GPU (got a ", t.device(),
              " tensor); this package has no CPU implementation of the hot path");
}

at::TensorOptions opts(const Tensor& like) { return like.options(); }
at::TensorOptions iopts(const Tensor& like) { return like.options().dtype(at::kInt); }

// ----------------------------------------------------------------------------- neighbour build
int strategy_code(const std::string& s) {
  if (s == "brute") return TMDNET_NL_BRUTE;
  if (s == "shared") return TMDNET_NL_SHARED;
  if (s == "cell") return TMDNET_NL_CELL;
  TORCH_CHECK(false, "Unknown kernel name");
}

// reference box checks (neighbors_cpu.cpp:35-56, common.cuh)
void validate_box(const double* v, double c) {
  TORCH_CHECK(v[1] == 0, "Invalid box vectors: box_vectors[0][1] != 0");
  TORCH_CHECK(v[2] == 0, "Invalid box vectors: box_vectors[0][2] != 0");
  TORCH_CHECK(v[5] == 0, "Invalid box vectors: box_vectors[1][2] != 0");
  TORCH_CHECK(v[0] >= 2 * c, "Invalid box vectors: box_vectors[0][0] < 2*cutoff");
  TORCH_CHECK(v[4] >= 2 * c, "Invalid box vectors: box_vectors[1][1] < 2*cutoff");
  TORCH_CHECK(v[8] >= 2 * c, "Invalid box vectors: box_vectors[2][2] < 2*cutoff");
  TORCH_CHECK(v[0] >= 2 * v[3], "Invalid box vectors: box_vectors[0][0] < 2*box_vectors[1][0]");
  TORCH_CHECK(v[0] >= 2 * v[6], "Invalid box vectors: box_vectors[0][0] < 2*box_vectors[1][0]");
  TORCH_CHECK(v[4] >= 2 * v[7], "Invalid box vectors: box_vectors[1][1] < 2*box_vectors[2][1]");
}

struct Built {
  Tensor nb, dl, dist, num, row_ptr, tr;
};

// One tmdnet_nl_build launch sequence (kernels.neighbor_pairs_raw's contract).
Built nl_build(const std::string& strategy_in, const Tensor& pos, const Tensor& batch, const Tensor& box,
               bool use_periodic, double cl, double cu, int64_t max_pairs, bool loop, bool include_transpose,
               bool pad, bool want_csr) {
  require_gpu(pos, "get_neighbor_pairs");
  TORCH_CHECK(pos.dim() == 2 && pos.size(1) == 3, "Expected \"positions\" to have two dimensions with size 3");
  TORCH_CHECK(pos.size(0) > 0, "Expected the 1nd dimension size of \"positions\" to be more than 0");
  TORCH_CHECK(pos.is_contiguous(), "Expected \"positions\" to be contiguous");
  TORCH_CHECK(batch.dim() == 1 && batch.size(0) == pos.size(0) && batch.scalar_type() == at::kLong &&
                  batch.is_contiguous() && batch.device() == pos.device(),
              "Expected \"batch\" to be a contiguous int64 vector matching \"positions\"");
  TORCH_CHECK(max_pairs > 0, "Expected \"max_num_neighbors\" to be positive");
  TORCH_CHECK(cu > 0, "Expected \"cutoff\" to be positive");
  const int n = static_cast<int>(pos.size(0));
  std::string strategy = strategy_in;
  int st = strategy_code(strategy);
  if (st == TMDNET_NL_BRUTE && n >= 32768) st = TMDNET_NL_SHARED;  // reference neighbors_cuda.cu:81-83
  double box9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  bool have_box = false;
  if ((use_periodic || st == TMDNET_NL_CELL) && box.defined() && box.numel() > 0) {
    TORCH_CHECK(box.dim() == 2 && box.size(0) == 3 && box.size(1) == 3,
                "Expected \"box_vectors\" to have shape (3, 3)");
    Tensor b = box.detach().to(at::kCPU).to(at::kDouble).contiguous();
    for (int i = 0; i < 9; ++i) box9[i] = b.data_ptr<double>()[i];
    have_box = true;
  }
  if (use_periodic) {
    TORCH_CHECK(have_box, "Expected \"box_vectors\" to have shape (3, 3)");
    validate_box(box9, cu);
  }
  if (st == TMDNET_NL_CELL) {
    TORCH_CHECK(have_box, "Expected \"box_size\" to have shape (3, 3)");
    TORCH_CHECK(box9[1] == 0 && box9[2] == 0 && box9[3] == 0 && box9[5] == 0 && box9[6] == 0 && box9[7] == 0,
                "Expected \"box_size\" to be diagonal");
  }
  const int cap = static_cast<int>(max_pairs);
  const double* bp = have_box ? box9 : nullptr;
  size_t ws_bytes = tmdnet_nl_workspace_bytes(n, st, bp, cu);
  Built B;
  Tensor ws = at::empty({static_cast<int64_t>(std::max<size_t>(ws_bytes, 16))}, pos.options().dtype(at::kByte));
  B.nb = at::empty({2, cap}, iopts(pos));
  B.dl = at::empty({cap, 3}, opts(pos));
  B.dist = at::empty({cap}, opts(pos));
  B.num = at::empty({1}, iopts(pos));
  if (want_csr) B.row_ptr = at::empty({n + 1}, iopts(pos));
  if (want_csr && include_transpose) B.tr = at::empty({cap}, iopts(pos));
  check(tmdnet_nl_build(dcode(pos), st, pos.data_ptr(), batch.data_ptr<int64_t>(), n, bp, use_periodic ? 1 : 0, cl,
                        cu, cap, loop ? 1 : 0, include_transpose ? 1 : 0, ptr<int32_t>(B.nb), ptr(B.dl),
                        ptr(B.dist), ptr<int32_t>(B.num), ptr<int32_t>(B.row_ptr), ptr<int32_t>(B.tr),
                        pad ? 1 : 0, ws.data_ptr(), static_cast<size_t>(ws.numel()), stream_of(pos)),
        "tmdnet_nl_build");
  return B;
}

// ----------------------------------------------------------------------------- raw op backward
// Second order of the raw op's backward: the derivative of the reference's index_add_ expression
// (neighbors_cuda.cu:50-68) written out in differentiable ATen ops.  Per edge slot (s -> t), valid
// when s >= 0 and r != 0:  w = gg[s] - gg[t];  d gd = w,  d gr = (dl.w)/r,  d dl = gr/r w,
// d r = -gr (dl.w)/r^2.
struct NlEdgesBwd : public Function<NlEdgesBwd> {
  static Tensor forward(AutogradContext* ctx, const Tensor& gd, const Tensor& gr, const Tensor& dl,
                        const Tensor& dist, const Tensor& nb, int64_t n) {
    Tensor gpos = at::empty({n, 3}, opts(dl));
    Tensor gd_ = contig(gd), gr_ = contig(gr);
    check(tmdnet_nl_backward_edges(dcode(dl), static_cast<int>(n), ptr<int32_t>(nb), static_cast<int>(dist.size(0)),
                                   ptr(gd_), ptr(gr_), ptr(dl), ptr(dist), ptr(gpos), stream_of(dl)),
          "tmdnet_nl_backward_edges");
    ctx->save_for_backward({gr_, dl, dist, nb});
    return gpos;
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Tensor gr = sv[0], dl = sv[1], dist = sv[2], nb = sv[3];
    Tensor gg = go[0];
    if (!gg.defined()) return {Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
    Tensor nbl = nb.to(at::kLong);
    Tensor s = nbl[0], t = nbl[1];
    Tensor valid = (s >= 0) & (t >= 0) & (dist != 0);
    Tensor inval = valid.logical_not();
    Tensor w = (gg.index_select(0, s.clamp_min(0)) - gg.index_select(0, t.clamp_min(0))) *
               valid.unsqueeze(1).to(dl.scalar_type());
    Tensor rs = dist.masked_fill(inval, 1);
    Tensor dlw = (dl * w).sum(1);
    Tensor d_gd = w;
    Tensor d_gr = dlw / rs;
    Tensor d_dl, d_r;
    if (gr.defined()) {
      Tensor grs = gr.masked_fill(inval, 0);
      d_dl = (grs / rs).unsqueeze(1) * w;
      d_r = -grs * dlw / (rs * rs);
    }
    return {d_gd, d_gr, d_dl, d_r, Tensor(), Tensor()};
  }
};

// torchmdnet_neighbors::get_neighbor_pairs with autograd (reference NeighborAutograd,
// neighbors_cuda.cu:25-72).  Returns (neighbors, deltas, distances, num_pairs) in the reference order.
struct NeighborPairs : public Function<NeighborPairs> {
  static variable_list forward(AutogradContext* ctx, const std::string& strategy, const Tensor& positions,
                               const Tensor& batch, const Tensor& box, bool use_periodic, double cl, double cu,
                               int64_t max_pairs, bool loop, bool include_transpose) {
    at::AutoDispatchBelowADInplaceOrView guard;
    Built B = nl_build(strategy, positions, batch, box, use_periodic, cl, cu, max_pairs, loop, include_transpose,
                       /*pad=*/true, /*want_csr=*/false);
    ctx->saved_data["n"] = positions.size(0);
    ctx->mark_non_differentiable({B.nb, B.num});
    ctx->save_for_backward({B.nb, B.dl, B.dist});  // outputs: saved without a reference cycle
    return {B.nb, B.dl, B.dist, B.num};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Tensor nb = sv[0], dl = sv[1], dist = sv[2];
    const int64_t n = ctx->saved_data["n"].toInt();
    Tensor gd = go[1], gr = go[2];
    Tensor none;
    if (!gd.defined() && !gr.defined())
      return {none, none, none, none, none, none, none, none, none, none};
    Tensor gpos = NlEdgesBwd::apply(gd, gr, dl, dist, nb, n);
    return {none, gpos, none, none, none, none, none, none, none, none};
  }
};

}  // namespace tmdt

namespace tmdt {

// ----------------------------------------------------------------------------- model-path graph
// Graph tensors travel as (row_ptr, src, dst, transpose); n = row_ptr.size(0) - 1, E = src.size(0).
struct G {
  Tensor row_ptr, src, dst, tr;
  int n() const { return static_cast<int>(row_ptr.size(0) - 1); }
  int E() const { return static_cast<int>(src.size(0)); }
};

G graph_of(AutogradContext* ctx, const char* prefix = "g") {
  G g;
  g.row_ptr = ctx->saved_data[std::string(prefix) + "_row_ptr"].toTensor();
  g.src = ctx->saved_data[std::string(prefix) + "_src"].toTensor();
  g.dst = ctx->saved_data[std::string(prefix) + "_dst"].toTensor();
  auto t = ctx->saved_data[std::string(prefix) + "_tr"];
  if (t.isTensor()) g.tr = t.toTensor();
  return g;
}

void keep_graph(AutogradContext* ctx, const G& g, const char* prefix = "g") {
  ctx->saved_data[std::string(prefix) + "_row_ptr"] = g.row_ptr;
  ctx->saved_data[std::string(prefix) + "_src"] = g.src;
  ctx->saved_data[std::string(prefix) + "_dst"] = g.dst;
  if (g.tr.defined()) ctx->saved_data[std::string(prefix) + "_tr"] = g.tr;
}

// Differentiable restatement of tmdnet_nl_backward2 (third order only): the gradient of
// <gg, nl_backward(pos, gd, gr)> w.r.t. (pos, gg, gr) (kernels.nl_backward2_composite).
variable_list nl_backward2_composite(const Tensor& pos, const Tensor& gg, const Tensor& gr, const Tensor& dl0,
                                     const Tensor& dist, const G& g) {
  const int64_t n = pos.size(0);
  Tensor s = g.src.to(at::kLong), d = g.dst.to(at::kLong);
  Tensor live = ((dist != 0) & (s >= 0) & (s < n) & (d >= 0) & (d < n)).to(pos.scalar_type()).unsqueeze(1);
  s = s.clamp(0, n - 1);
  d = d.clamp(0, n - 1);
  Tensor shift = (dl0 - (pos.index_select(0, s) - pos.index_select(0, d))).detach();
  Tensor dl = pos.index_select(0, s) - pos.index_select(0, d) + shift;
  Tensor r = at::where(dist == 0, at::ones_like(dist), (dl * dl).sum(1)).sqrt();
  Tensor u = dl / r.unsqueeze(1);
  Tensor w = (gg.index_select(0, s) - gg.index_select(0, d)) * live;
  Tensor uw = (u * w).sum(1, true);
  Tensor d_pos = at::zeros_like(pos);
  if (gr.defined()) {
    Tensor h = (gr / r).unsqueeze(1) * (w - u * uw);
    d_pos = d_pos.index_add(0, s, h).index_add(0, d, -h);
  }
  return {d_pos, w, uw.squeeze(1)};
}

struct NlGeomBwd2 : public Function<NlGeomBwd2> {
  // (pos, gg, gd?, gr?, dl, dist) -> (d_pos, d_gd, d_gr): tmdnet_nl_backward2
  static variable_list forward(AutogradContext* ctx, const Tensor& pos, const Tensor& gg, const Tensor& gd,
                               const Tensor& gr, const Tensor& dl, const Tensor& dist, const Tensor& row_ptr,
                               const Tensor& src, const Tensor& dst, const Tensor& tr) {
    G g{row_ptr, src, dst, tr};
    const int cap = g.E();
    Tensor d_pos = at::empty_like(pos);
    Tensor d_gd = gd.defined() ? at::empty({cap, 3}, opts(pos)) : Tensor();
    Tensor d_gr = gr.defined() ? at::empty({cap}, opts(pos)) : Tensor();
    Tensor ggc = gg.contiguous();
    check(tmdnet_nl_backward2(dcode(pos), g.n(), ptr<int32_t>(row_ptr), ptr<int32_t>(src), ptr<int32_t>(tr), cap,
                              ptr(gr), ptr(dl), ptr(dist), ptr(ggc), ptr(d_pos), ptr(d_gd), ptr(d_gr),
                              stream_of(pos)),
          "tmdnet_nl_backward2");
    keep_graph(ctx, g);
    ctx->save_for_backward({pos, ggc, gr, dl, dist});
    if (!d_gd.defined()) d_gd = at::zeros({0}, opts(pos));
    if (!d_gr.defined()) d_gr = at::zeros({0}, opts(pos));
    return {d_pos, d_gd, d_gr};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Tensor pos = sv[0], gg = sv[1], gr = sv[2], dl = sv[3], dist = sv[4];
    G g = graph_of(ctx);
    const bool create = at::GradMode::is_enabled();
    variable_list res(10);
    at::AutoGradMode enable(true);
    Tensor p = pos.detach().requires_grad_(true);
    Tensor g_ = gg.detach().requires_grad_(true);
    Tensor r_ = gr.defined() ? gr.detach().requires_grad_(true) : Tensor();
    auto outs = nl_backward2_composite(p, g_, r_, dl.detach(), dist.detach(), g);
    variable_list os, gs;
    for (int i = 0; i < 3; ++i)
      if (go[i].defined() && go[i].numel() == outs[i].numel()) {
        os.push_back(outs[i]);
        gs.push_back(go[i]);
      }
    if (os.empty()) return res;
    variable_list ins = {p, g_};
    if (r_.defined()) ins.push_back(r_);
    auto grads = torch::autograd::grad(os, ins, gs, true, create, true);
    res[0] = grads[0];
    res[1] = grads[1];
    if (r_.defined()) res[3] = grads[2];
    return res;
  }
};

struct NlGeomBwd : public Function<NlGeomBwd> {
  // (pos, gd?, gr?, dl, dist) -> gpos: tmdnet_nl_backward (CSR, transpose map, no atomics)
  static Tensor forward(AutogradContext* ctx, const Tensor& pos, const Tensor& gd, const Tensor& gr, const Tensor& dl,
                        const Tensor& dist, const Tensor& row_ptr, const Tensor& src, const Tensor& dst,
                        const Tensor& tr) {
    G g{row_ptr, src, dst, tr};
    Tensor gpos = at::empty_like(pos);
    Tensor gd_ = contig(gd), gr_ = contig(gr);
    check(tmdnet_nl_backward(dcode(pos), g.n(), ptr<int32_t>(row_ptr), ptr<int32_t>(tr), g.E(), ptr(gd_), ptr(gr_),
                             ptr(dl), ptr(dist), ptr(gpos), stream_of(pos)),
          "tmdnet_nl_backward");
    keep_graph(ctx, g);
    ctx->save_for_backward({pos, gd_, gr_, dl, dist});
    return gpos;
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Tensor pos = sv[0], gd = sv[1], gr = sv[2], dl = sv[3], dist = sv[4];
    G g = graph_of(ctx);
    variable_list res(9);
    if (!go[0].defined()) return res;
    auto o = NlGeomBwd2::apply(pos, go[0], gd, gr, dl, dist, g.row_ptr, g.src, g.dst, g.tr);
    res[0] = o[0];
    if (gd.defined()) res[1] = o[1];
    if (gr.defined()) res[2] = o[2];
    return res;  // dl / dist are functions of pos: their dependence is inside d_pos
  }
};

// tmdnet::neighbor_graph: the symmetric CSR list of the fused model path (kernels.build_graph).
// static_capacity > 0: every per-edge output has that many rows, no host synchronisation (HIP-graph
// capturable; num_pairs > capacity is reported on the device through num_pairs).  Otherwise the
// list is trimmed to the pairs found (one host sync, reference resize_to_fit) and an overflow of
// max_num_pairs raises when check_errors.
struct NeighborGraph : public Function<NeighborGraph> {
  static variable_list forward(AutogradContext* ctx, const Tensor& pos, const Tensor& batch, const Tensor& box,
                               bool use_periodic, double cl, double cu, int64_t max_pairs, bool loop,
                               const std::string& strategy, bool check_errors, int64_t static_capacity) {
    at::AutoDispatchBelowADInplaceOrView guard;
    const bool stat = static_capacity > 0;
    const int64_t cap = stat ? static_capacity : max_pairs;
    Tensor bx = box;
    if (strategy == "cell" && !use_periodic) {  // reference utils.py:199-202: a 3 x cutoff box
      const double l = 3.0 * cu;
      bx = at::zeros({3, 3}, at::TensorOptions().dtype(at::kDouble));
      bx[0][0] = l;
      bx[1][1] = l;
      bx[2][2] = l;
    }
    Built B = nl_build(strategy, pos, batch, bx, use_periodic, cl, cu, cap, loop, true, /*pad=*/true,
                       /*want_csr=*/true);
    Tensor src = B.nb[0], dst = B.nb[1], tr = B.tr, dl = B.dl, dist = B.dist;
    bool symmetric = true;
    if (!stat) {
      const int64_t found = B.num.item<int>();  // host sync (reference resize_to_fit)
      TORCH_CHECK(!check_errors || found <= cap, "Found num_pairs(", found, ") > max_num_pairs(", cap, ")");
      const int64_t E = std::min(found, cap);
      symmetric = found <= cap;
      src = src.narrow(0, 0, E);
      dst = dst.narrow(0, 0, E);
      tr = tr.narrow(0, 0, E);
      dl = dl.narrow(0, 0, E);
      dist = dist.narrow(0, 0, E);
    }
    ctx->saved_data["symmetric"] = symmetric;
    G g{B.row_ptr, src, dst, tr};
    keep_graph(ctx, g);
    ctx->save_for_backward({pos, dl, dist});
    ctx->mark_non_differentiable({B.row_ptr, src, dst, tr, B.num});
    return {B.row_ptr, src, dst, tr, dl, dist, B.num};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Tensor pos = sv[0], dl = sv[1], dist = sv[2];
    variable_list res(11);
    Tensor gd = go[4], gr = go[5];
    if (!gd.defined() && !gr.defined()) return res;
    TORCH_CHECK(ctx->saved_data["symmetric"].toBool(),
                "torchmd-net_amd: the neighbour backward needs the full symmetric list (num_pairs exceeded "
                "max_num_pairs)");
    G g = graph_of(ctx);
    res[0] = NlGeomBwd::apply(pos, gd, gr, dl, dist, g.row_ptr, g.src, g.dst, g.tr);
    return res;
  }
};

// ----------------------------------------------------------------------------- edge geometry
Tensor cos_cut(const Tensor& r, double cl, double cu) {
  if (cl > 0) {
    Tensor c = 0.5 * (at::cos(M_PI * (2 * (r - cl) / (cu - cl) + 1.0)) + 1.0);
    return c * (r < cu).to(r.scalar_type()) * (r > cl).to(r.scalar_type());
  }
  return 0.5 * (at::cos(r * (M_PI / cu)) + 1.0) * (r < cu).to(r.scalar_type());
}

// kernels._edge_geom_composite: (f, C, u) in ATen ops (reference utils.py:298-344, 368-390)
variable_list edge_geom_composite(const Tensor& dl, const Tensor& dist, const Tensor& selfmask, const Tensor& mu,
                                  const Tensor& beta, double cl, double cu, int64_t rbf, bool wf, bool wc, bool wu) {
  variable_list out(3);
  if (wf) {
    Tensor r = dist.unsqueeze(-1);
    if (rbf == TMDNET_RBF_EXPNORM) {
      const double alpha = 5.0 / (cu - cl);
      out[0] = cos_cut(r, 0.0, cu) * at::exp(-beta * (at::exp(alpha * (-r + cl)) - mu).pow(2));
    } else {
      out[0] = at::exp(beta[0] * (r - mu).pow(2));
    }
  }
  if (wc) out[1] = cos_cut(dist, cl, cu);
  if (wu) {
    Tensor sq = (dl * dl).sum(1);
    Tensor nrm = at::where(selfmask, at::ones_like(sq), sq).sqrt().unsqueeze(1);
    out[2] = at::where(selfmask.unsqueeze(1), dl, dl / nrm);
  }
  return out;
}

struct Geo {
  double cl, cu;
  int64_t rbf;
};

Geo geo_of(AutogradContext* ctx) {
  return {ctx->saved_data["cl"].toDouble(), ctx->saved_data["cu"].toDouble(), ctx->saved_data["rbf"].toInt()};
}

void keep_geo(AutogradContext* ctx, double cl, double cu, int64_t rbf) {
  ctx->saved_data["cl"] = cl;
  ctx->saved_data["cu"] = cu;
  ctx->saved_data["rbf"] = rbf;
}

struct EdgeGeomBwd : public Function<EdgeGeomBwd> {
  // (dl, dist, gf?, gC?, gu?) -> (g_dl, g_r): tmdnet_edge_geom_bwd
  static variable_list forward(AutogradContext* ctx, const Tensor& dl, const Tensor& dist, const Tensor& gf,
                               const Tensor& gC, const Tensor& gu, const Tensor& src, const Tensor& dst,
                               const Tensor& mu, const Tensor& beta, double cl, double cu, int64_t rbf) {
    const int E = static_cast<int>(dist.size(0));
    Tensor g_r = at::empty_like(dist), g_dl = at::empty_like(dl);
    Tensor gf_ = contig(gf), gC_ = contig(gC), gu_ = contig(gu);
    check(tmdnet_edge_geom_bwd(dcode(dist), E, static_cast<int>(mu.size(0)), static_cast<int>(rbf), ptr<int32_t>(src),
                               ptr<int32_t>(dst), ptr(dl), ptr(dist), ptr(mu), ptr(beta), cl, cu, ptr(gf_), ptr(gC_),
                               ptr(gu_), ptr(g_r), ptr(g_dl), stream_of(dist)),
          "tmdnet_edge_geom_bwd");
    keep_geo(ctx, cl, cu, rbf);
    ctx->save_for_backward({dl, dist, gf_, gC_, gu_, src, dst, mu, beta});
    return {g_dl, g_r};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Tensor dl = sv[0], dist = sv[1], src = sv[5], dst = sv[6], mu = sv[7], beta = sv[8];
    Tensor ups[3] = {sv[2], sv[3], sv[4]};
    Geo c = geo_of(ctx);
    const bool create = at::GradMode::is_enabled();
    variable_list res(12);
    at::AutoGradMode enable(true);
    Tensor dl_ = dl.detach().requires_grad_(true), r_ = dist.detach().requires_grad_(true);
    Tensor u_[3];
    for (int i = 0; i < 3; ++i) u_[i] = ups[i].defined() ? ups[i].detach().requires_grad_(true) : Tensor();
    auto outs = edge_geom_composite(dl_, r_, src == dst, mu, beta, c.cl, c.cu, c.rbf, u_[0].defined(),
                                    u_[1].defined(), u_[2].defined());
    variable_list os, gs;
    for (int i = 0; i < 3; ++i)
      if (u_[i].defined()) {
        os.push_back(outs[i]);
        gs.push_back(u_[i]);
      }
    auto first = torch::autograd::grad(os, {dl_, r_}, gs, true, true, true);
    variable_list fs, fg;
    for (int i = 0; i < 2; ++i)
      if (first[i].defined() && go[i].defined() && first[i].requires_grad()) {
        fs.push_back(first[i]);
        fg.push_back(go[i]);
      }
    if (fs.empty()) return res;
    variable_list ins = {dl_, r_};
    for (int i = 0; i < 3; ++i)
      if (u_[i].defined()) ins.push_back(u_[i]);
    auto second = torch::autograd::grad(fs, ins, fg, true, create, true);
    res[0] = second[0];
    res[1] = second[1];
    int k = 2;
    for (int i = 0; i < 3; ++i)
      if (u_[i].defined()) res[2 + i] = second[k++];
    return res;
  }
};

struct EdgeGeom : public Function<EdgeGeom> {
  static variable_list forward(AutogradContext* ctx, const Tensor& dl, const Tensor& dist, const Tensor& src,
                               const Tensor& dst, const Tensor& mu, const Tensor& beta, double cl, double cu,
                               int64_t rbf, bool want_rbf) {
    require_gpu(dist, "edge_geometry");
    const int E = static_cast<int>(dist.size(0));
    const int R = static_cast<int>(mu.size(0));
    Tensor f = want_rbf ? at::empty({E, R}, opts(dist)) : at::zeros({0}, opts(dist));
    Tensor C = at::empty({E}, opts(dist));
    Tensor u = at::empty({E, 3}, opts(dist));
    check(tmdnet_edge_geom_fwd(dcode(dist), E, R, static_cast<int>(rbf), ptr<int32_t>(src), ptr<int32_t>(dst),
                               ptr(dl), ptr(dist), ptr(mu), ptr(beta), cl, cu, want_rbf ? ptr(f) : nullptr,
                               ptr(C), ptr(u), stream_of(dist)),
          "tmdnet_edge_geom_fwd");
    keep_geo(ctx, cl, cu, rbf);
    ctx->saved_data["want_rbf"] = want_rbf;
    ctx->save_for_backward({dl, dist, src, dst, mu, beta});
    if (!want_rbf) ctx->mark_non_differentiable({f});
    return {f, C, u};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    Geo c = geo_of(ctx);
    Tensor gf = ctx->saved_data["want_rbf"].toBool() ? go[0] : Tensor();
    variable_list res(10);
    if (!gf.defined() && !go[1].defined() && !go[2].defined()) return res;
    auto o = EdgeGeomBwd::apply(sv[0], sv[1], gf, go[1], go[2], sv[2], sv[3], sv[4], sv[5], c.cl, c.cu, c.rbf);
    res[0] = o[0];
    res[1] = o[1];
    return res;
  }
};

// ----------------------------------------------------------------------------- neighbour embedding
Tensor nbr_embed_composite(const Tensor& x, const Tensor& w, const Tensor& C, const G& g) {
  Tensor s = g.src.to(at::kLong), d = g.dst.to(at::kLong);
  Tensor keep = ((s != d) & (s >= 0)).to(x.scalar_type()).unsqueeze(1);
  s = s.clamp_min(0);
  d = d.clamp_min(0);
  Tensor m = x.index_select(0, s) * (w * C.unsqueeze(1)) * keep;
  return at::zeros({g.n(), x.size(1)}, opts(x)).index_add(0, d, m);
}

struct NbrEmbedBwd : public Function<NbrEmbedBwd> {
  static variable_list forward(AutogradContext* ctx, const Tensor& gout, const Tensor& x, const Tensor& w,
                               const Tensor& C, const Tensor& row_ptr, const Tensor& src, const Tensor& dst) {
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(x.size(0)), H = static_cast<int>(x.size(1)), E = g.E();
    Tensor go = gout.contiguous();
    Tensor gx = at::empty({N, H}, opts(x));
    Tensor gw = at::zeros({E, H}, opts(x)), gC = at::zeros({E}, opts(x));
    check(tmdnet_nbr_embed_bwd(dcode(x), N, H, ptr<int32_t>(row_ptr), ptr<int32_t>(src), E, ptr(x), ld(x), ptr(w),
                               ld(w), ptr(C), ptr(go), ld(go), ptr(gx), ptr(gw), ptr(gC), stream_of(x)),
          "tmdnet_nbr_embed_bwd");
    keep_graph(ctx, g);
    ctx->save_for_backward({go, x, w, C});
    return {gx, gw, gC};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    const bool create = at::GradMode::is_enabled();
    variable_list res(7);
    at::AutoGradMode enable(true);
    variable_list leaves;
    for (int i = 0; i < 4; ++i) leaves.push_back(sv[i].detach().requires_grad_(true));
    Tensor out = nbr_embed_composite(leaves[1], leaves[2], leaves[3], g);
    auto first = torch::autograd::grad({out}, {leaves[1], leaves[2], leaves[3]}, {leaves[0]}, true, true, true);
    variable_list fs, fg;
    for (int i = 0; i < 3; ++i)
      if (go[i].defined() && first[i].defined()) {
        fs.push_back(first[i]);
        fg.push_back(go[i]);
      }
    if (fs.empty()) return res;
    auto second = torch::autograd::grad(fs, leaves, fg, true, create, true);
    for (int i = 0; i < 4; ++i) res[i] = second[i];
    return res;
  }
};

struct NbrEmbed : public Function<NbrEmbed> {
  static Tensor forward(AutogradContext* ctx, const Tensor& x_in, const Tensor& w_in, const Tensor& C_in,
                        const Tensor& row_ptr, const Tensor& src, const Tensor& dst) {
    require_gpu(x_in, "nbr_embed");
    Tensor x = rowmajor(x_in), w = rowmajor(w_in), C = C_in.contiguous();
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(x.size(0)), H = static_cast<int>(x.size(1));
    TORCH_CHECK(w.size(0) == g.E() && w.size(1) == H && C.size(0) == g.E(), "nbr_embed: shape mismatch");
    Tensor out = at::empty({N, H}, opts(x));
    check(tmdnet_nbr_embed_fwd(dcode(x), N, H, ptr<int32_t>(row_ptr), ptr<int32_t>(src), g.E(), ptr(x), ld(x), ptr(w),
                               ld(w), ptr(C), ptr(out), H, nullptr, nullptr, stream_of(x)),
          "tmdnet_nbr_embed_fwd");
    keep_graph(ctx, g);
    ctx->save_for_backward({x, w, C});
    return out;
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    variable_list res(6);
    if (!go[0].defined()) return res;
    auto o = NbrEmbedBwd::apply(go[0], sv[0], sv[1], sv[2], g.row_ptr, g.src, g.dst);
    res[0] = o[0];
    res[1] = o[1];
    res[2] = o[2];
    return res;
  }
};

// ----------------------------------------------------------------------------- ET message
struct EtMsgBwd : public Function<EtMsgBwd> {
  // (gx, gvec, q, k, v, vec?, pk?, pv?, C, u) -> (gq, gk, gv, gvec_in, gpk, gpv, gC, gu): tmdnet_et_message_bwd;
  // its backward is tmdnet_et_message_bwd2 (the third order is not provided)
  static variable_list forward(AutogradContext* ctx, const Tensor& gx, const Tensor& gvec, const Tensor& q,
                               const Tensor& k, const Tensor& v, const Tensor& vec, const Tensor& pk, const Tensor& pv,
                               const Tensor& C, const Tensor& u, const Tensor& row_ptr, const Tensor& src,
                               const Tensor& dst, int64_t heads) {
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(q.size(0)), H = static_cast<int>(q.size(1)), E = g.E();
    Tensor gq = at::empty({N, H}, opts(q)), gk = at::empty({N, H}, opts(q)), gv = at::empty({N, 3 * H}, opts(q));
    Tensor gw = at::empty({N, 3, H}, opts(q));
    Tensor gpk = pk.defined() ? at::empty({E, H}, opts(q)) : at::zeros({0}, opts(q));
    Tensor gpv = pv.defined() ? at::empty({E, 3 * H}, opts(q)) : at::zeros({0}, opts(q));
    Tensor gC = at::empty({E}, opts(q)), gu = at::empty({E, 3}, opts(q));
    Tensor gxc = gx.contiguous(), gvc = gvec.contiguous();
    check(tmdnet_et_message_bwd(dcode(q), N, H, static_cast<int>(heads), ptr<int32_t>(row_ptr), ptr<int32_t>(src), E,
                                ptr(q), ld(q), ptr(k), ld(k), ptr(v), ld(v), ptr(vec), ptr(pk), ld(pk), ptr(pv),
                                ld(pv), ptr(C), ptr(u), ptr(gxc), ptr(gvc), ptr(gq), ptr(gk), ptr(gv),
                                vec.defined() ? ptr(gw) : nullptr, pk.defined() ? ptr(gpk) : nullptr,
                                pv.defined() ? ptr(gpv) : nullptr, ptr(gC), ptr(gu), nullptr, nullptr, nullptr, 0,
                                nullptr, nullptr, stream_of(q)),
          "tmdnet_et_message_bwd");
    if (!vec.defined()) gw.zero_();
    keep_graph(ctx, g);
    ctx->saved_data["heads"] = heads;
    ctx->save_for_backward({gxc, gvc, q, k, v, vec, pk, pv, C, u});
    return {gq, gk, gv, gw, gpk, gpv, gC, gu};
  }

  static variable_list backward(AutogradContext* ctx, variable_list gg) {
    auto sv = ctx->get_saved_variables();
    Tensor gx = sv[0], gvec = sv[1], q = sv[2], k = sv[3], v = sv[4], vec = sv[5], pk = sv[6], pv = sv[7], C = sv[8],
           u = sv[9];
    G g = graph_of(ctx);
    const int heads = static_cast<int>(ctx->saved_data["heads"].toInt());
    const int N = static_cast<int>(q.size(0)), H = static_cast<int>(q.size(1)), E = g.E();
    auto o = opts(q);
    auto dense = [&](const Tensor& t, at::IntArrayRef shape) {
      return (!t.defined() || t.numel() == 0) ? at::zeros(shape, o) : t.contiguous();
    };
    Tensor ggq = dense(gg[0], {N, H}), ggk = dense(gg[1], {N, H}), ggv = dense(gg[2], {N, 3 * H});
    Tensor ggw = dense(gg[3], {N, 3, H});
    Tensor ggpk = pk.defined() ? dense(gg[4], {E, H}) : Tensor();
    Tensor ggpv = pv.defined() ? dense(gg[5], {E, 3 * H}) : Tensor();
    Tensor ggC = dense(gg[6], {E}), ggu = dense(gg[7], {E, 3});
    Tensor d_gx = at::empty({N, H}, o), d_gvec = at::empty({N, 3, H}, o), d_q = at::empty({N, H}, o);
    Tensor d_k = at::zeros({N, H}, o), d_v = at::zeros({N, 3 * H}, o), d_vec = at::zeros({N, 3, H}, o);
    Tensor d_pk = pk.defined() ? at::empty({E, H}, o) : Tensor();
    Tensor d_pv = pv.defined() ? at::empty({E, 3 * H}, o) : Tensor();
    Tensor d_C = at::empty({E}, o), d_u = at::empty({E, 3}, o);
    check(tmdnet_et_message_bwd2(dcode(q), N, H, heads, ptr<int32_t>(g.row_ptr), ptr<int32_t>(g.src), E, ptr(q), ld(q),
                                 ptr(k), ld(k), ptr(v), ld(v), ptr(vec), ptr(pk), ld(pk), ptr(pv), ld(pv), ptr(C),
                                 ptr(u), ptr(gx), ptr(gvec), ptr(ggq), ptr(ggk), ptr(ggv), ptr(ggw), ptr(ggpk),
                                 ld(ggpk), ptr(ggpv), ld(ggpv), ptr(ggC), ptr(ggu), ptr(d_gx), ptr(d_gvec), ptr(d_q),
                                 ptr(d_k), ptr(d_v), vec.defined() ? ptr(d_vec) : nullptr, ptr(d_pk), ptr(d_pv),
                                 ptr(d_C), ptr(d_u), 0, stream_of(q)),
          "tmdnet_et_message_bwd2");
    return {d_gx, d_gvec, d_q, d_k, d_v, vec.defined() ? d_vec : Tensor(), d_pk, d_pv, d_C, d_u,
            Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

struct EtMsg : public Function<EtMsg> {
  static variable_list forward(AutogradContext* ctx, const Tensor& q_in, const Tensor& k_in, const Tensor& v_in,
                               const Tensor& vec_in, const Tensor& pk_in, const Tensor& pv_in, const Tensor& C_in,
                               const Tensor& u_in, const Tensor& row_ptr, const Tensor& src, const Tensor& dst,
                               int64_t heads) {
    require_gpu(q_in, "et_message");
    Tensor q = rowmajor(q_in), k = rowmajor(k_in), v = rowmajor(v_in), pk = rowmajor(pk_in), pv = rowmajor(pv_in);
    Tensor vec = contig(vec_in), C = C_in.contiguous(), u = u_in.contiguous();
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(q.size(0)), H = static_cast<int>(q.size(1));
    TORCH_CHECK(heads > 0 && H % heads == 0, "et_message: hidden channels must divide into heads");
    TORCH_CHECK(k.sizes() == q.sizes() && v.size(0) == N && v.size(1) == 3 * H, "et_message: q/k/v shapes");
    TORCH_CHECK(!vec.defined() || (vec.size(0) == N && vec.size(1) == 3 && vec.size(2) == H), "et_message: vec shape");
    TORCH_CHECK(C.size(0) == g.E() && u.size(0) == g.E(), "et_message: per-edge shapes");
    TORCH_CHECK(!pk.defined() || (pk.size(0) == g.E() && pk.size(1) == H), "et_message: dk shape");
    TORCH_CHECK(!pv.defined() || (pv.size(0) == g.E() && pv.size(1) == 3 * H), "et_message: dv shape");
    Tensor xo = at::empty({N, H}, opts(q)), vo = at::empty({N, 3, H}, opts(q));
    check(tmdnet_et_message_fwd(dcode(q), N, H, static_cast<int>(heads), ptr<int32_t>(row_ptr), ptr<int32_t>(src),
                                g.E(), ptr(q), ld(q), ptr(k), ld(k), ptr(v), ld(v), ptr(vec), ptr(pk), ld(pk), ptr(pv),
                                ld(pv), ptr(C), ptr(u), ptr(xo), ptr(vo), 0, nullptr, nullptr, stream_of(q)),
          "tmdnet_et_message_fwd");
    keep_graph(ctx, g);
    ctx->saved_data["heads"] = heads;
    ctx->save_for_backward({q, k, v, vec, pk, pv, C, u});
    return {xo, vo};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    const int64_t heads = ctx->saved_data["heads"].toInt();
    Tensor q = sv[0];
    const int64_t N = q.size(0), H = q.size(1);
    Tensor gx = go[0].defined() ? go[0] : at::zeros({N, H}, opts(q));
    Tensor gvec = go[1].defined() ? go[1] : at::zeros({N, 3, H}, opts(q));
    auto o = EtMsgBwd::apply(gx, gvec, sv[0], sv[1], sv[2], sv[3], sv[4], sv[5], sv[6], sv[7], g.row_ptr, g.src, g.dst,
                             heads);
    variable_list res(12);
    res[0] = o[0];
    res[1] = o[1];
    res[2] = o[2];
    if (sv[3].defined()) res[3] = o[3];
    if (sv[4].defined()) res[4] = o[4];
    if (sv[5].defined()) res[5] = o[5];
    res[6] = o[6];
    res[7] = o[7];
    return res;
  }
};

// ----------------------------------------------------------------------------- TensorNet edge ops
// Compact component-major tensors [9][N][H] (include/tmdnet.h).  self0_mult: multiplicity of atom 0's
// self loop (the reference CUDA static_shapes padding, tensornet.py:215-221; 1 = none).
Tensor self0_weight(const G& g, const Tensor& like, double m) {
  Tensor w = at::ones({g.E()}, opts(like));
  if (m != 1.0) w = at::where((g.src == 0) & (g.dst == 0), at::full_like(w, m), w);
  return w;
}

Tensor skew_c(const Tensor& u) {  // (a01, a02, a12) of skew(u)
  return at::stack({-u.select(1, 2), u.select(1, 1), -u.select(1, 0)}, 1);
}

Tensor sym_c(const Tensor& u) {  // (s00, s11, s01, s02, s12) of u u^T - |u|^2/3 Id
  Tensor tr = (u * u).sum(1) / 3;
  Tensor x = u.select(1, 0), y = u.select(1, 1), z = u.select(1, 2);
  return at::stack({x * x - tr, y * y - tr, x * y, x * z, y * z}, 1);
}

// kernels.tn_embed_composite (tensornet.py:295-315, scatter to edge_index[0])
Tensor tn_embed_composite(const Tensor& P, const Tensor& Q, const Tensor& W, const Tensor& C, const Tensor& u,
                          const G& g, double m) {
  Tensor valid = (g.src >= 0).to(P.scalar_type());
  Tensor s = g.src.to(at::kLong).clamp_min(0), d = g.dst.to(at::kLong).clamp_min(0);
  const int64_t H = P.size(1), N = g.n();
  Tensor wt = (self0_weight(g, C, m) * C * valid).unsqueeze(1);
  Tensor z = (P.index_select(0, s) + Q.index_select(0, d)) * wt;
  Tensor W1 = W.narrow(1, 0, H), W2 = W.narrow(1, H, H), W3 = W.narrow(1, 2 * H, H);
  std::vector<Tensor> coef = {z * W1};
  Tensor a = skew_c(u), sy = sym_c(u);
  Tensor zw2 = z * W2, zw3 = z * W3;
  for (int k = 0; k < 3; ++k) coef.push_back(zw2 * a.select(1, k).unsqueeze(1));
  for (int k = 0; k < 5; ++k) coef.push_back(zw3 * sy.select(1, k).unsqueeze(1));
  std::vector<Tensor> rows;
  Tensor zero = at::zeros({N, H}, opts(P));
  for (auto& c : coef) rows.push_back(zero.index_add(0, s, c));
  return at::stack(rows, 0);
}

// kernels.tn_message_composite (tensornet.py:329-332: gather edge_index[1], scatter edge_index[0])
Tensor tn_message_composite(const Tensor& ea, const Tensor& Tc, const G& g, double m) {
  Tensor valid = (g.src >= 0).to(Tc.scalar_type());
  Tensor s = g.src.to(at::kLong).clamp_min(0), d = g.dst.to(at::kLong).clamp_min(0);
  const int64_t N = Tc.size(1), H = Tc.size(2);
  Tensor f = ea.reshape({-1, H, 3}) * (self0_weight(g, ea, m) * valid).view({-1, 1, 1});
  Tensor zero = at::zeros({N, H}, opts(Tc));
  std::vector<Tensor> rows;
  for (int k = 0; k < 9; ++k) {
    const int part = k == 0 ? 0 : (k < 4 ? 1 : 2);
    rows.push_back(zero.index_add(0, s, f.select(2, part) * Tc[k].index_select(0, d)));
  }
  return at::stack(rows, 0);
}

// second order by recompute: gradients of <ggs, VJP(composite, primals, gouts)> w.r.t. (gouts, primals)
template <class F>
variable_list double_backward(F&& fwd, const variable_list& saved_gouts, const variable_list& saved_primals,
                              const variable_list& ggs) {
  const bool create = at::GradMode::is_enabled();
  at::AutoGradMode enable(true);
  variable_list go, pr, leaves;
  for (auto& t : saved_gouts) go.push_back(t.detach().requires_grad_(true));
  for (auto& t : saved_primals) pr.push_back(t.detach().requires_grad_(true));
  leaves = go;
  leaves.insert(leaves.end(), pr.begin(), pr.end());
  Tensor out = fwd(pr);
  auto first = torch::autograd::grad({out}, pr, {go[0]}, true, true, true);
  variable_list fs, fg;
  for (size_t i = 0; i < first.size() && i < ggs.size(); ++i)
    if (ggs[i].defined() && first[i].defined()) {
      fs.push_back(first[i]);
      fg.push_back(ggs[i]);
    }
  if (fs.empty()) return variable_list(leaves.size());
  return torch::autograd::grad(fs, leaves, fg, true, create, true);
}

struct TnEmbedBwd : public Function<TnEmbedBwd> {
  static variable_list forward(AutogradContext* ctx, const Tensor& gE, const Tensor& P, const Tensor& Q,
                               const Tensor& W, const Tensor& C, const Tensor& u, const Tensor& row_ptr,
                               const Tensor& src, const Tensor& dst, double m) {
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(P.size(0)), H = static_cast<int>(P.size(1)), E = g.E();
    auto o = opts(P);
    Tensor gEc = gE.contiguous();
    Tensor gP = at::empty({N, H}, o), gQ = at::empty({N, H}, o), gW = at::empty({E, 3 * H}, o);
    Tensor gC = at::empty({E}, o), gu = at::empty({E, 3}, o);
    check(tmdnet_tn_embed_bwd(dcode(P), N, H, ptr<int32_t>(row_ptr), ptr<int32_t>(src), E, m, nullptr, 0, ptr(P),
                              ptr(Q), ptr(W), ld(W), ptr(C), ptr(u), ptr(gEc), ptr(gP), ptr(gQ), ptr(gW), ptr(gC),
                              ptr(gu), stream_of(P)),
          "tmdnet_tn_embed_bwd");
    keep_graph(ctx, g);
    ctx->saved_data["m"] = m;
    ctx->save_for_backward({gEc, P, Q, W, C, u});
    return {gP, gQ, gW, gC, gu};
  }

  static variable_list backward(AutogradContext* ctx, variable_list ggs) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    const double m = ctx->saved_data["m"].toDouble();
    auto r = double_backward(
        [&](const variable_list& p) { return tn_embed_composite(p[0], p[1], p[2], p[3], p[4], g, m); }, {sv[0]},
        {sv[1], sv[2], sv[3], sv[4], sv[5]}, ggs);
    variable_list res(10);
    for (int i = 0; i < 6; ++i) res[i] = r[i];
    return res;
  }
};

struct TnEmbed : public Function<TnEmbed> {
  static Tensor forward(AutogradContext* ctx, const Tensor& P_in, const Tensor& Q_in, const Tensor& W_in,
                        const Tensor& C_in, const Tensor& u_in, const Tensor& row_ptr, const Tensor& src,
                        const Tensor& dst, double m) {
    require_gpu(P_in, "tn_embed");
    Tensor P = P_in.contiguous(), Q = Q_in.contiguous(), W = rowmajor(W_in), C = C_in.contiguous(),
           u = u_in.contiguous();
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(P.size(0)), H = static_cast<int>(P.size(1));
    TORCH_CHECK(Q.sizes() == P.sizes() && W.size(0) == g.E() && W.size(1) == 3 * H && C.size(0) == g.E() &&
                    u.size(0) == g.E(),
                "tn_embed: shape mismatch");
    Tensor out = at::empty({9, N, H}, opts(P));
    check(tmdnet_tn_embed_fwd(dcode(P), N, H, ptr<int32_t>(row_ptr), ptr<int32_t>(src), g.E(), m, nullptr, 0, ptr(P),
                              ptr(Q), ptr(W), ld(W), ptr(C), ptr(u), ptr(out), stream_of(P)),
          "tmdnet_tn_embed_fwd");
    keep_graph(ctx, g);
    ctx->saved_data["m"] = m;
    ctx->save_for_backward({P, Q, W, C, u});
    return out;
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    variable_list res(9);
    if (!go[0].defined()) return res;
    auto o = TnEmbedBwd::apply(go[0], sv[0], sv[1], sv[2], sv[3], sv[4], g.row_ptr, g.src, g.dst,
                               ctx->saved_data["m"].toDouble());
    for (int i = 0; i < 5; ++i) res[i] = o[i];
    return res;
  }
};

struct TnMessageBwd : public Function<TnMessageBwd> {
  static variable_list forward(AutogradContext* ctx, const Tensor& gmsg, const Tensor& ea, const Tensor& Tc,
                               const Tensor& row_ptr, const Tensor& src, const Tensor& dst, double m) {
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(Tc.size(1)), H = static_cast<int>(Tc.size(2)), E = g.E();
    Tensor gm = gmsg.contiguous();
    Tensor gea = at::empty({E, 3 * H}, opts(Tc)), gT = at::empty_like(Tc);
    check(tmdnet_tn_message_bwd(dcode(Tc), N, H, ptr<int32_t>(row_ptr), ptr<int32_t>(src), E, m, nullptr, 0, ptr(ea),
                                ld(ea), ptr(Tc), ptr(gm), ptr(gea), ptr(gT), stream_of(Tc)),
          "tmdnet_tn_message_bwd");
    keep_graph(ctx, g);
    ctx->saved_data["m"] = m;
    ctx->save_for_backward({gm, ea, Tc});
    return {gea, gT};
  }

  static variable_list backward(AutogradContext* ctx, variable_list ggs) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    const double m = ctx->saved_data["m"].toDouble();
    auto r = double_backward([&](const variable_list& p) { return tn_message_composite(p[0], p[1], g, m); },
                             {sv[0]}, {sv[1], sv[2]}, ggs);
    variable_list res(7);
    for (int i = 0; i < 3; ++i) res[i] = r[i];
    return res;
  }
};

struct TnMessage : public Function<TnMessage> {
  static Tensor forward(AutogradContext* ctx, const Tensor& ea_in, const Tensor& Tc_in, const Tensor& row_ptr,
                        const Tensor& src, const Tensor& dst, double m) {
    require_gpu(Tc_in, "tn_message");
    Tensor ea = rowmajor(ea_in), Tc = Tc_in.contiguous();
    G g{row_ptr, src, dst, Tensor()};
    const int N = static_cast<int>(Tc.size(1)), H = static_cast<int>(Tc.size(2));
    TORCH_CHECK(Tc.size(0) == 9 && ea.size(0) == g.E() && ea.size(1) == 3 * H, "tn_message: shape mismatch");
    Tensor msg = at::empty_like(Tc);
    check(tmdnet_tn_message_fwd(dcode(Tc), N, H, ptr<int32_t>(row_ptr), ptr<int32_t>(src), g.E(), m, nullptr, 0,
                                ptr(ea), ld(ea), ptr(Tc), ptr(msg), stream_of(Tc)),
          "tmdnet_tn_message_fwd");
    keep_graph(ctx, g);
    ctx->saved_data["m"] = m;
    ctx->save_for_backward({ea, Tc});
    return msg;
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    G g = graph_of(ctx);
    variable_list res(6);
    if (!go[0].defined()) return res;
    auto o = TnMessageBwd::apply(go[0], sv[0], sv[1], g.row_ptr, g.src, g.dst, ctx->saved_data["m"].toDouble());
    res[0] = o[0];
    res[1] = o[1];
    return res;
  }
};

Tensor tn_embed(const Tensor& P, const Tensor& Q, const Tensor& W, const Tensor& C, const Tensor& u,
                const Tensor& row_ptr, const Tensor& src, const Tensor& dst, double self0_mult) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(P.device());
  return TnEmbed::apply(P, Q, W, C, u, row_ptr, src, dst, self0_mult);
}

Tensor tn_message(const Tensor& ea, const Tensor& Tc, const Tensor& row_ptr, const Tensor& src, const Tensor& dst,
                  double self0_mult) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(ea.device());
  return TnMessage::apply(ea, Tc, row_ptr, src, dst, self0_mult);
}

// ----------------------------------------------------------------------------- op entry points
std::tuple<Tensor, Tensor, Tensor, Tensor> get_neighbor_pairs_fwd(const std::string& strategy, const Tensor& positions,
                                                                  const Tensor& batch, const Tensor& box_vectors,
                                                                  bool use_periodic, const at::Scalar& cutoff_lower,
                                                                  const at::Scalar& cutoff_upper,
                                                                  const at::Scalar& max_num_pairs, bool loop,
                                                                  bool include_transpose) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(positions.device());
  Built B = nl_build(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower.toDouble(),
                     cutoff_upper.toDouble(), max_num_pairs.toLong(), loop, include_transpose, true, false);
  return {B.nb, B.dl, B.dist, B.num};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> get_neighbor_pairs_autograd(
    const std::string& strategy, const Tensor& positions, const Tensor& batch, const Tensor& box_vectors,
    bool use_periodic, const at::Scalar& cutoff_lower, const at::Scalar& cutoff_upper, const at::Scalar& max_num_pairs,
    bool loop, bool include_transpose) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(positions.device());
  auto r = NeighborPairs::apply(strategy, positions, batch, box_vectors, use_periodic, cutoff_lower.toDouble(),
                                cutoff_upper.toDouble(), max_num_pairs.toLong(), loop, include_transpose);
  return {r[0], r[1], r[2], r[3]};
}

std::tuple<Tensor, Tensor, Tensor, Tensor> get_neighbor_pairs_cpu(const std::string&, const Tensor&, const Tensor&,
                                                                  const Tensor&, bool, const at::Scalar&,
                                                                  const at::Scalar&, const at::Scalar&, bool, bool) {
  TORCH_CHECK(false, "torchmd-net_amd: get_neighbor_pairs runs only on a ROCm GPU (CPU tensors given)");
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> neighbor_graph(
    const Tensor& pos, const Tensor& batch, const c10::optional<Tensor>& box, bool use_periodic, double cutoff_lower,
    double cutoff_upper, int64_t max_num_pairs, bool loop, const std::string& strategy, bool check_errors,
    int64_t static_capacity) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(pos.device());
  auto r = NeighborGraph::apply(pos, batch, box.has_value() ? *box : Tensor(), use_periodic, cutoff_lower, cutoff_upper,
                                max_num_pairs, loop, strategy, check_errors, static_capacity);
  return {r[0], r[1], r[2], r[3], r[4], r[5], r[6]};
}

std::tuple<Tensor, Tensor, Tensor> edge_geometry(const Tensor& deltas, const Tensor& distances, const Tensor& src,
                                                 const Tensor& dst, const Tensor& mu, const Tensor& beta,
                                                 double cutoff_lower, double cutoff_upper, int64_t rbf_type,
                                                 bool want_rbf) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(distances.device());
  auto r = EdgeGeom::apply(deltas, distances, src, dst, mu.detach().to(distances.scalar_type()).contiguous(),
                           beta.detach().to(distances.scalar_type()).contiguous(), cutoff_lower, cutoff_upper,
                           rbf_type, want_rbf);
  return {r[0], r[1], r[2]};
}

Tensor nbr_embed(const Tensor& x, const Tensor& w, const Tensor& C, const Tensor& row_ptr, const Tensor& src,
                 const Tensor& dst) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(x.device());
  return NbrEmbed::apply(x, w, C, row_ptr, src, dst);
}

std::tuple<Tensor, Tensor> et_message(const Tensor& q, const Tensor& k, const Tensor& v,
                                      const c10::optional<Tensor>& vec, const c10::optional<Tensor>& pk,
                                      const c10::optional<Tensor>& pv, const Tensor& C, const Tensor& u,
                                      const Tensor& row_ptr, const Tensor& src, const Tensor& dst, int64_t heads) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(q.device());
  auto r = EtMsg::apply(q, k, v, vec.has_value() ? *vec : Tensor(), pk.has_value() ? *pk : Tensor(),
                        pv.has_value() ? *pv : Tensor(), C, u, row_ptr, src, dst, heads);
  return {r[0], r[1]};
}

}  // namespace tmdt

// The reference schema, verbatim (torchmdnet/neighbors/neighbors.cpp:3-5).
TORCH_LIBRARY(torchmdnet_neighbors, m) {
  m.def("get_neighbor_pairs(str strategy, Tensor positions, Tensor batch, Tensor box_vectors, bool use_periodic, "
        "Scalar cutoff_lower, Scalar cutoff_upper, Scalar max_num_pairs, bool loop, bool include_transpose) -> "
        "(Tensor neighbors, Tensor distances, Tensor distance_vecs, Tensor num_pairs)");
}

TORCH_LIBRARY_IMPL(torchmdnet_neighbors, CUDA, m) { m.impl("get_neighbor_pairs", tmdt::get_neighbor_pairs_fwd); }
TORCH_LIBRARY_IMPL(torchmdnet_neighbors, AutogradCUDA, m) {
  m.impl("get_neighbor_pairs", tmdt::get_neighbor_pairs_autograd);
}
TORCH_LIBRARY_IMPL(torchmdnet_neighbors, CPU, m) { m.impl("get_neighbor_pairs", tmdt::get_neighbor_pairs_cpu); }

// The fused model path's operators (TorchScript-visible).  Registered as CompositeImplicitAutograd
// entry points: each wraps its own C++ autograd Function, and each Function's forward checks that its
// tensors live on the GPU.
TORCH_LIBRARY(tmdnet, m) {
  m.def("neighbor_graph(Tensor pos, Tensor batch, Tensor? box, bool use_periodic, float cutoff_lower, "
        "float cutoff_upper, int max_num_pairs, bool loop, str strategy, bool check_errors, int static_capacity) -> "
        "(Tensor row_ptr, Tensor src, Tensor dst, Tensor transpose, Tensor deltas, Tensor distances, "
        "Tensor num_pairs)");
  m.def("edge_geometry(Tensor deltas, Tensor distances, Tensor src, Tensor dst, Tensor mu, Tensor beta, "
        "float cutoff_lower, float cutoff_upper, int rbf_type, bool want_rbf) -> (Tensor rbf, Tensor cutoff, "
        "Tensor unit)");
  m.def("nbr_embed(Tensor x, Tensor w, Tensor cutoff, Tensor row_ptr, Tensor src, Tensor dst) -> Tensor");
  m.def("et_message(Tensor q, Tensor k, Tensor v, Tensor? vec, Tensor? pk, Tensor? pv, Tensor cutoff, Tensor unit, "
        "Tensor row_ptr, Tensor src, Tensor dst, int heads) -> (Tensor x, Tensor vec)");
  m.def("tn_embed(Tensor P, Tensor Q, Tensor W, Tensor cutoff, Tensor unit, Tensor row_ptr, Tensor src, "
        "Tensor dst, float self0_mult) -> Tensor");
  m.def("tn_message(Tensor edge_attr, Tensor comp, Tensor row_ptr, Tensor src, Tensor dst, float self0_mult) -> "
        "Tensor");
}

TORCH_LIBRARY_IMPL(tmdnet, CompositeImplicitAutograd, m) {
  m.impl("neighbor_graph", tmdt::neighbor_graph);
  m.impl("edge_geometry", tmdt::edge_geometry);
  m.impl("nbr_embed", tmdt::nbr_embed);
  m.impl("et_message", tmdt::et_message);
  m.impl("tn_embed", tmdt::tn_embed);
  m.impl("tn_message", tmdt::tn_message);
}
