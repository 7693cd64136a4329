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
#include <torch/custom_class.h>
#include <torch/library.h>

#include <cmath>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

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

// Optional tensor arguments of the autograd Functions: an absent input must be an EMPTY optional
// (no autograd edge) -- an undefined Tensor argument would be recorded as an input without metadata.
using OptT = c10::optional<Tensor>;
OptT opt(const Tensor& t) { return t.defined() ? OptT(t) : OptT(); }
Tensor val(const OptT& t) { return (t.has_value() && t->defined()) ? *t : Tensor(); }

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
  // (absent vec / pk / pv travel as empty optionals: no autograd edge, so the Function stays
  // recordable under create_graph)
  static variable_list forward(AutogradContext* ctx, const Tensor& gx, const Tensor& gvec, const Tensor& q,
                               const Tensor& k, const Tensor& v, const OptT& vec_o, const OptT& pk_o,
                               const OptT& pv_o, const Tensor& C, const Tensor& u, const Tensor& row_ptr,
                               const Tensor& src, const Tensor& dst, int64_t heads, int64_t acts) {
    const Tensor vec = val(vec_o), pk = val(pk_o), pv = val(pv_o);
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
                                pv.defined() ? ptr(gpv) : nullptr, ptr(gC), ptr(gu), nullptr, nullptr, nullptr,
                                static_cast<int>(acts), nullptr, nullptr, stream_of(q)),
          "tmdnet_et_message_bwd");
    if (!vec.defined()) gw.zero_();
    keep_graph(ctx, g);
    ctx->saved_data["heads"] = heads;
    ctx->saved_data["acts"] = acts;
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
                                 ptr(d_C), ptr(d_u), static_cast<int>(ctx->saved_data["acts"].toInt()), stream_of(q)),
          "tmdnet_et_message_bwd2");
    return {d_gx, d_gvec, d_q, d_k, d_v, vec.defined() ? d_vec : Tensor(), d_pk, d_pv, d_C, d_u,
            Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

struct EtMsg : public Function<EtMsg> {
  static variable_list forward(AutogradContext* ctx, const Tensor& q_in, const Tensor& k_in, const Tensor& v_in,
                               const OptT& vec_o, const OptT& pk_o, const OptT& pv_o, const Tensor& C_in,
                               const Tensor& u_in, const Tensor& row_ptr, const Tensor& src, const Tensor& dst,
                               int64_t heads, int64_t acts) {
    const Tensor vec_in = val(vec_o), pk_in = val(pk_o), pv_in = val(pv_o);
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
                                ld(pv), ptr(C), ptr(u), ptr(xo), ptr(vo), static_cast<int>(acts), nullptr, nullptr,
                                stream_of(q)),
          "tmdnet_et_message_fwd");
    keep_graph(ctx, g);
    ctx->saved_data["heads"] = heads;
    ctx->saved_data["acts"] = acts;
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
    auto o = EtMsgBwd::apply(gx, gvec, sv[0], sv[1], sv[2], opt(sv[3]), opt(sv[4]), opt(sv[5]), sv[6], sv[7], g.row_ptr,
                             g.src, g.dst,
                             heads, ctx->saved_data["acts"].toInt());
    variable_list res(13);
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
                                      const Tensor& row_ptr, const Tensor& src, const Tensor& dst, int64_t heads,
                                      int64_t acts) {
  // launches, allocations and the stream on the input's device whatever the caller's current device
  // (the autograd engine runs each backward on its device's thread with that device current)
  const c10::OptionalDeviceGuard guard(q.device());
  auto r = EtMsg::apply(q, k, v, opt(val(vec)), opt(val(pk)), opt(val(pv)), C, u, row_ptr, src, dst, heads, acts);
  return {r[0], r[1]};
}

// ----------------------------------------------------------------------------- ET layer stack
// tmdnet::et_stack: every EquivariantMultiHeadAttention layer of TorchMD_ET plus the model's out_norm
// (reference torchmd_et.py:177-187, 272-347) as ONE operator, so a TorchScript'd model runs the same
// fused launches as the eager stack (et_stack.py) instead of the per-layer ATen loop:
//   forward:  all layers' dk/dv projections in one GEMM (tmdnet_proj_f32 over the edges), per layer one
//             grouped GEMM ([q|k|v] + vec_proj, tmdnet_gemm_f32), tmdnet_et_message_fwd, the o_proj GEMM
//             and the epilogue fused with the next layer's LayerNorm (tmdnet_et_epilogue_ln_fwd; the
//             last one with out_norm);
//   backward (a force evaluation: no parameter gradient requested): "dr mode" -- d(dk,dv)/dr formed
//             once (tmdnet_rbf_deriv + one projection GEMM), contracted with the projection gradient
//             inside tmdnet_et_message_bwd, accumulating d/d r per edge; per layer the epilogue / o_proj /
//             message / grouped transposed GEMM / LayerNorm backward kernels;
//   parameter gradients (training through TorchScript) and every higher order: autograd over the
//             differentiable restatement (ATen Linears / LayerNorms + the tmdnet::et_message Function,
//             itself HIP to second order).
// f must be rbf(dist) with the fixed (non-trainable) basis given by (mu, beta, rbf_type): the
// operator's gradient for f is delivered to dist (f gets none), as the eager stack's dr mode does.
// fp32 only (the model falls back to the per-layer loop for fp64 or a trainable basis).
struct StackCfg {
  int64_t heads, rbf;
  double cl, cu;
  bool hk, hv, out_norm;
  int64_t acts;  // TMDNET_ET_ACT bits of the layers' activations
};

void keep_cfg(AutogradContext* ctx, const StackCfg& c) {
  ctx->saved_data["heads"] = c.heads;
  ctx->saved_data["rbf"] = c.rbf;
  ctx->saved_data["cl"] = c.cl;
  ctx->saved_data["cu"] = c.cu;
  ctx->saved_data["flags"] = int64_t(c.hk) | (int64_t(c.hv) << 1) | (int64_t(c.out_norm) << 2);
  ctx->saved_data["acts"] = c.acts;
}

StackCfg cfg_of(AutogradContext* ctx) {
  const int64_t fl = ctx->saved_data["flags"].toInt();
  return {ctx->saved_data["heads"].toInt(), ctx->saved_data["rbf"].toInt(), ctx->saved_data["cl"].toDouble(),
          ctx->saved_data["cu"].toDouble(), bool(fl & 1), bool(fl & 2), bool(fl & 4),
          ctx->saved_data["acts"].toInt()};
}

constexpr double kLnEps = 1e-5;  // nn.LayerNorm default (reference torchmd_et.py:223, :117)

int64_t stack_np(bool hk, bool hv) { return 11 + 2 * int64_t(hk) + 2 * int64_t(hv); }

// Large-row fp32 GEMM on tmdnet_gemm_x3_f32 (kernels.gemm_x3): B split per call (a [N][K] weight with
// trans_b, a [K][N] right operand without); false when outside its envelope
bool gemm_x3_into(const Tensor& A, const Tensor& B, bool trans_b, const Tensor& bias, const Tensor& C, bool beta) {
  const int M = static_cast<int>(A.size(0)), N = static_cast<int>(C.size(1)), K = static_cast<int>(A.size(1));
  auto al = [](const Tensor& t) { return !t.defined() || reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  if (!(A.scalar_type() == at::kFloat && B.scalar_type() == at::kFloat && C.scalar_type() == at::kFloat && M > 0 &&
        K % 32 == 0 && N % 16 == 0 && A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1 &&
        A.stride(0) % 4 == 0 && B.stride(0) % 4 == 0 && C.stride(0) % 4 == 0 && al(A) && al(B) && al(C) &&
        (!bias.defined() || (bias.is_contiguous() && al(bias)))))
    return false;
  void* st = stream_of(A);
  // (a split launch per call, as kernels.X3_WSPLIT = "launch": faster at C5 than the in-kernel split of
  // tmdnet_gemm_x3w_f32, and nothing cached)
  Tensor bp = at::empty({3, N, K}, A.options().dtype(at::kShort));
  int rc = trans_b ? tmdnet_proj_split_f32(N, K, B.data_ptr(), static_cast<int>(B.stride(0)), bp.data_ptr(), st)
                   : tmdnet_split_t_f32(N, K, B.data_ptr(), static_cast<int>(B.stride(0)), bp.data_ptr(), st);
  if (rc == TMDNET_UNSUPPORTED) return false;
  check(rc, "tmdnet_split");
  rc = tmdnet_gemm_x3_f32(M, N, K, A.data_ptr(), static_cast<int>(A.stride(0)), bp.data_ptr(),
                          bias.defined() ? bias.data_ptr() : nullptr, C.data_ptr(), static_cast<int>(C.stride(0)),
                          beta ? 1 : 0, st);
  if (rc == TMDNET_UNSUPPORTED) return false;
  check(rc, "tmdnet_gemm_x3_f32");
  return true;
}

// C = A op(B) (+ bias) (+ C if beta) on the hand-written grouped GEMM (up to 16384 rows) or the x3 GEMM
// (more rows), the library outside both envelopes
void gemm_into(const Tensor& A, const Tensor& B, bool trans_b, const Tensor& bias, const Tensor& C, bool beta) {
  const int M = static_cast<int>(A.size(0)), N = static_cast<int>(C.size(1)), K = static_cast<int>(A.size(1));
  if (M > 16384 && gemm_x3_into(A, B, trans_b, bias, C, beta)) return;
  if (A.scalar_type() == at::kFloat && M > 0 && M <= 16384 && A.stride(1) == 1 && B.stride(1) == 1 &&
      C.stride(1) == 1) {
    int dims[8] = {M, N, K, static_cast<int>(A.stride(0)), static_cast<int>(B.stride(0)),
                   static_cast<int>(C.stride(0)), int(trans_b), int(beta)};
    const void* ptrs[4] = {A.data_ptr(), B.data_ptr(), bias.defined() ? bias.data_ptr() : nullptr, C.data_ptr()};
    const int rc = tmdnet_gemm_f32(1, dims, ptrs, stream_of(A));
    if (rc != TMDNET_UNSUPPORTED) {
      check(rc, "tmdnet_gemm_f32");
      return;
    }
  }
  Tensor Bop = trans_b ? B.t() : B;
  if (beta) {
    C.addmm_(A, Bop);
    if (bias.defined()) C.add_(bias);
  } else if (bias.defined()) {
    at::addmm_out(const_cast<Tensor&>(C), bias, A, Bop);
  } else {
    at::mm_out(const_cast<Tensor&>(C), A, Bop);
  }
}

// Two independent products in ONE tmdnet_gemm_f32 launch when both fit the grouped kernel (the layer's
// [q|k|v]^T and vec_proj^T input gradients: 8 launches fewer per C2 force pass); else two gemm_into
void gemm2_into(const Tensor& A1, const Tensor& B1, bool tb1, const Tensor& C1, bool beta1, const Tensor& A2,
                const Tensor& B2, bool tb2, const Tensor& C2, bool beta2) {
  auto ok = [](const Tensor& A, const Tensor& B, const Tensor& C) {
    return A.scalar_type() == at::kFloat && A.size(0) > 0 && A.size(0) <= 16384 && A.stride(1) == 1 &&
           B.stride(1) == 1 && C.stride(1) == 1;
  };
  if (ok(A1, B1, C1) && ok(A2, B2, C2)) {
    int dims[16];
    const void* ptrs[8];
    const Tensor* As[2] = {&A1, &A2};
    const Tensor* Bs[2] = {&B1, &B2};
    const Tensor* Cs[2] = {&C1, &C2};
    const bool tb[2] = {tb1, tb2}, be[2] = {beta1, beta2};
    for (int i = 0; i < 2; ++i) {
      const Tensor &A = *As[i], &B = *Bs[i], &C = *Cs[i];
      const int d[8] = {static_cast<int>(A.size(0)), static_cast<int>(C.size(1)), static_cast<int>(A.size(1)),
                        static_cast<int>(A.stride(0)), static_cast<int>(B.stride(0)), static_cast<int>(C.stride(0)),
                        int(tb[i]), int(be[i])};
      for (int j = 0; j < 8; ++j) dims[8 * i + j] = d[j];
      ptrs[4 * i] = A.data_ptr();
      ptrs[4 * i + 1] = B.data_ptr();
      ptrs[4 * i + 2] = nullptr;
      ptrs[4 * i + 3] = C.data_ptr();
    }
    const int rc = tmdnet_gemm_f32(2, dims, ptrs, stream_of(A1));
    if (rc != TMDNET_UNSUPPORTED) {
      check(rc, "tmdnet_gemm_f32");
      return;
    }
  }
  gemm_into(A1, B1, tb1, Tensor(), C1, beta1);
  gemm_into(A2, B2, tb2, Tensor(), C2, beta2);
}

// out = A W^T (+ bias) for the dk/dv projection (tmdnet_proj_f32 on the exact bf16 split; library otherwise)
void proj_into(const Tensor& A, const Tensor& W, const Tensor& Wp, const Tensor& bias, const Tensor& out) {
  const int M = static_cast<int>(A.size(0)), N = static_cast<int>(W.size(0)), K = static_cast<int>(W.size(1));
  if (Wp.defined() && M > 0) {
    const int rc = tmdnet_proj_f32(M, N, K, A.data_ptr(), static_cast<int>(A.stride(0)), Wp.data_ptr(),
                                   static_cast<long long>(N) * K, bias.defined() ? bias.data_ptr() : nullptr,
                                   out.data_ptr(), static_cast<int>(out.stride(0)), stream_of(A));
    if (rc != TMDNET_UNSUPPORTED) {
      check(rc, "tmdnet_proj_f32");
      return;
    }
  }
  if (bias.defined()) at::addmm_out(const_cast<Tensor&>(out), bias, A, W.t());
  else at::mm_out(const_cast<Tensor&>(out), A, W.t());
}

// The stacked weights of one parameter set: per layer [q|k|v] (5H x H) and its bias, all layers' [dk; dv]
// rows (L*D x R) + bias and their bf16 split.  Formed on EVERY call -- there is no cache that an in-place
// write could leave stale (a fused optimizer step, `p.data.copy_`, an EMA swap: none bumps a version
// counter that a cache could key on).  The Python stack (et_stack.py _stack_views) makes the parameters
// row blocks of one buffer in exactly this layout, and TorchMD_ET stacks them before it calls this operator
// (eager eval and __prepare_scriptable__), so the stacked weights are VIEWS of the parameters' own storage:
// no copy, always current.  Parameters stored separately (e.g. after `.to()` of a scripted module) are
// concatenated per call.  The dk/dv weights' bf16 split is one launch per call.
struct Packed {
  std::vector<Tensor> qkv_w, qkv_b;
  Tensor dkv_w, dkv_b, dkv_wp;
};

// ts as consecutive row blocks of one storage (same dtype / device / trailing shape, contiguous, adjacent):
// that span as one tensor (a view); otherwise their concatenation (a copy)
static Tensor stacked_or_cat(const std::vector<Tensor>& ts) {
  const Tensor& a = ts[0];
  const int64_t row = a.dim() > 1 ? a.numel() / std::max<int64_t>(a.size(0), 1) : 1;
  bool ok = a.is_contiguous();
  int64_t rows = 0;
  for (const auto& t : ts) {
    ok = ok && t.is_contiguous() && t.dim() == a.dim() && t.scalar_type() == a.scalar_type() &&
         t.device() == a.device() && t.storage().unsafeGetStorageImpl() == a.storage().unsafeGetStorageImpl() &&
         t.storage_offset() == a.storage_offset() + rows * row;
    for (int64_t d = 1; ok && d < a.dim(); ++d) ok = t.size(d) == a.size(d);
    if (!ok) break;
    rows += t.size(0);
  }
  if (!ok) return at::cat(ts, 0).contiguous();
  std::vector<int64_t> sz(a.sizes().begin(), a.sizes().end());
  sz[0] = rows;
  return a.as_strided(sz, a.strides(), a.storage_offset());
}

void et_stack_invalidate() {}  // (kept for callers of the old cached form: nothing is cached any more)

std::shared_ptr<Packed> pack_stack(const std::vector<Tensor>& P, int64_t L, int64_t np, bool hk, bool hv) {
  auto pk = std::make_shared<Packed>();
  at::NoGradGuard ng;
  std::vector<Tensor> dw, db;
  for (int64_t l = 0; l < L; ++l) {
    const Tensor* p = P.data() + l * np;
    pk->qkv_w.push_back(stacked_or_cat({p[2], p[4], p[6]}));
    pk->qkv_b.push_back(stacked_or_cat({p[3], p[5], p[7]}));
    int64_t i = 11;
    if (hk) { dw.push_back(p[i]); db.push_back(p[i + 1]); i += 2; }
    if (hv) { dw.push_back(p[i]); db.push_back(p[i + 1]); }
  }
  if (!dw.empty()) {
    pk->dkv_w = stacked_or_cat(dw);
    pk->dkv_b = stacked_or_cat(db);
    const int N = static_cast<int>(pk->dkv_w.size(0)), K = static_cast<int>(pk->dkv_w.size(1));
    if (pk->dkv_w.scalar_type() == at::kFloat && (K == 32 || K == 64) && N % 16 == 0) {
      Tensor wp = at::empty({3, N, K}, pk->dkv_w.options().dtype(at::kShort));
      const int rc = tmdnet_proj_split_f32(N, K, pk->dkv_w.data_ptr(), K, wp.data_ptr(), stream_of(pk->dkv_w));
      if (rc != TMDNET_UNSUPPORTED) {
        check(rc, "tmdnet_proj_split_f32");
        pk->dkv_wp = wp;
      }
    }
  }
  return pk;
}

// The forward's intermediates the first-order backward reads (per layer, as et_stack._forward_layers);
// kept in the autograd context as an IValue capsule (freed with the graph).
struct StackActs : torch::CustomClassHolder {
  std::vector<Tensor> x, vec, xn, mean, rstd, qkv, vecp, xa, o;
  Tensor pkv_all, x_pre, mean_o, rstd_o;
  std::shared_ptr<Packed> pk;
  bool batched = true;
};

// differentiable restatement: (x, dist, C, u, params) -> (x_out, vec_out), the reference layer loop
std::pair<Tensor, Tensor> stack_composite(const Tensor& x_in, const Tensor& dist, const Tensor& C, const Tensor& u,
                                          const Tensor& mu, const Tensor& beta, const std::vector<Tensor>& P,
                                          const G& g, const StackCfg& c) {
  const int64_t H = x_in.size(1), np = stack_np(c.hk, c.hv);
  const int64_t L = (static_cast<int64_t>(P.size()) - (c.out_norm ? 2 : 0)) / np;
  Tensor f = edge_geom_composite(Tensor(), dist, Tensor(), mu, beta, c.cl, c.cu, c.rbf, true, false, false)[0];
  Tensor x = x_in, vec;
  for (int64_t l = 0; l < L; ++l) {
    const Tensor* p = P.data() + l * np;
    Tensor xn = at::layer_norm(x, {H}, p[0], p[1], kLnEps);
    Tensor q = at::linear(xn, p[2], p[3]), k = at::linear(xn, p[4], p[5]), v = at::linear(xn, p[6], p[7]);
    int64_t i = 11;
    Tensor pk, pv;
    if (c.hk) { pk = at::linear(f, p[i], p[i + 1]); i += 2; }
    if (c.hv) pv = at::linear(f, p[i], p[i + 1]);
    auto m = EtMsg::apply(q, k, v, opt(vec), opt(pk), opt(pv), C, u, g.row_ptr, g.src, g.dst, c.heads, c.acts);
    auto o = at::linear(m[0], p[9], p[10]).split(H, 1);
    if (vec.defined()) {
      auto vp = at::linear(vec, p[8]).split(H, -1);
      Tensor vec_dot = (vp[0] * vp[1]).sum(1);
      x = x + vec_dot * o[1] + o[2];
      vec = vec + vp[2] * o[0].unsqueeze(1) + m[1];
    } else {  // layer 0: vec = 0 (torchmd_et.py:176)
      x = x + o[2];
      vec = m[1];
    }
  }
  if (c.out_norm) x = at::layer_norm(x, {H}, P[P.size() - 2], P[P.size() - 1], kLnEps);
  return {x, vec};
}

// The node-fused layer mixes (et_nodemix.hip; et_stack.NODE_FUSE): LayerNorm + [q|k|v] + vec_proj, o_proj +
// the epilogue, and in the force pass the LayerNorm / epilogue backward + the o_proj input gradient, each one
// launch.  Used in the regime of the small grouped GEMM (3N <= 16384 rows; the x3 GEMMs above) at H = 128.
bool node_fuse_ok(int64_t N, int64_t H) { return H == 128 && N > 0 && 3 * N <= 16384; }

void ln_mix(const Tensor& x, const Tensor& ln_w, const Tensor& ln_b, const Tensor& w, const Tensor& b,
            const Tensor& vec, const Tensor& vec_w, const Tensor& qkv, Tensor* vecp, Tensor* xn, Tensor* mean,
            Tensor* rstd) {
  const int64_t N = x.size(0), H = x.size(1);
  auto o = opts(x);
  *xn = at::empty({N, H}, o);
  *mean = at::empty({N, 1}, o);
  *rstd = at::empty({N, 1}, o);
  *vecp = vec.defined() ? at::empty({N, 3, vec_w.size(0)}, o) : Tensor();
  check(tmdnet_et_ln_mix_f32(static_cast<int>(N), static_cast<int>(H), ptr(x), ptr(ln_w), ptr(ln_b), kLnEps, ptr(w),
                             ptr(b), static_cast<int>(w.size(0)), ptr(qkv), ptr(*xn), ptr(*mean), ptr(*rstd), ptr(vec),
                             vec.defined() ? ptr(vec_w) : nullptr, vec.defined() ? static_cast<int>(vec_w.size(0)) : 0,
                             ptr(*vecp), stream_of(x)),
        "tmdnet_et_ln_mix_f32");
}

void oproj_epi(const Tensor& xa, const Tensor& o_w, const Tensor& o_b, const Tensor& x, const Tensor& vec,
               const Tensor& vecp, const Tensor& veca, const Tensor& oo, Tensor* xo, Tensor* vo) {
  const int64_t N = x.size(0), H = x.size(1);
  *xo = at::empty({N, H}, opts(x));
  *vo = at::empty({N, 3, H}, opts(x));
  check(tmdnet_et_oproj_epilogue_f32(static_cast<int>(N), static_cast<int>(H), ptr(xa), ptr(o_w), ptr(o_b), ptr(x),
                                     ptr(vec), ptr(vecp), ptr(veca), ptr(oo), ptr(*xo), ptr(*vo), stream_of(x)),
        "tmdnet_et_oproj_epilogue_f32");
}

// returns g_x; g_xa (layer l-1's o_proj input gradient) into *g_xa
Tensor lnbwd_oproj(const Tensor& g_xn, const Tensor& x, const Tensor& mean, const Tensor& rstd, const Tensor& ln_w,
                   const Tensor& g_res, const Tensor& g_vec, const Tensor& vecp, const Tensor& oo, const Tensor& o_w,
                   const Tensor& g_vecp, const Tensor& g_o, Tensor* g_xa) {
  Tensor gx = at::empty_like(x);
  *g_xa = at::empty_like(x);
  check(tmdnet_et_lnbwd_oproj_f32(static_cast<int>(x.size(0)), static_cast<int>(x.size(1)), ptr(g_xn), ptr(x),
                                  ptr(mean), ptr(rstd), ptr(ln_w), ptr(g_res), ptr(g_vec), ptr(vecp), ptr(oo), ptr(o_w),
                                  ptr(gx), ptr(g_vecp), ptr(g_o), ptr(*g_xa), stream_of(x)),
        "tmdnet_et_lnbwd_oproj_f32");
  return gx;
}

// The fast first-order backward of a force evaluation (et_stack._backward_layers with dr=True):
// returns (g_x, g_dist, g_C, g_u).
variable_list stack_backward_dr(const StackActs& A, Tensor gX, Tensor gV, const Tensor& dist, const Tensor& C,
                                const Tensor& u, const Tensor& mu, const Tensor& beta, const std::vector<Tensor>& P,
                                const G& g, const StackCfg& c) {
  const int64_t N = gX.size(0), H = gX.size(1), E = g.E(), np = stack_np(c.hk, c.hv);
  const int64_t L = static_cast<int64_t>(A.x.size()), D = (int64_t(c.hk) + 3 * int64_t(c.hv)) * H;
  const bool has_e = c.hk || c.hv;
  auto o = opts(gX);
  // the edge gradients are accumulated across layers by the kernels; the first layer of the backward
  // overwrites them (separate tensors: they are outputs of the backward Function)
  Tensor g_C = at::empty({E}, o), g_u = at::empty({E, 3}, o), g_r = at::empty({E}, o);
  if (!has_e) g_r.zero_();
  Tensor dpkv_all;
  if (has_e) {  // d(dk,dv)/dr = (d f / d r) W^T, every layer in one GEMM (or per layer for large graphs)
    const int R = static_cast<int>(mu.size(0));
    Tensor fdp = at::empty({E, R}, o);
    check(tmdnet_rbf_deriv(dcode(dist), R, static_cast<int>(c.rbf), ptr(dist), ptr(mu), ptr(beta), c.cl, c.cu,
                           nullptr, static_cast<int>(E), ptr(fdp), stream_of(dist)),
          "tmdnet_rbf_deriv");
    if (A.batched) {
      dpkv_all = at::empty({E, L * D}, o);
      proj_into(fdp, A.pk->dkv_w, A.pk->dkv_wp, Tensor(), dpkv_all);
    } else {
      dpkv_all = fdp;  // per layer below
    }
  }
  std::vector<Tensor> g_o(L), g_vecp(L);
  for (int64_t l = 0; l < L; ++l) {
    g_o[l] = at::empty({N, 3 * H}, o);
    if (A.vec[l].defined()) g_vecp[l] = at::empty({N, 3, 3 * H}, o);
  }
  bool epi_done = false;
  const bool nf = node_fuse_ok(N, H);
  Tensor g_xa_pre;  // the next (lower) layer's g_xa, formed by the node-fused LayerNorm backward
  if (c.out_norm && nf) {  // back through out_norm, the last layer's epilogue and its o_proj^T in one kernel
    gX = lnbwd_oproj(gX, A.x_pre, A.mean_o, A.rstd_o, P[P.size() - 2], Tensor(), gV, A.vecp[L - 1], A.o[L - 1],
                     P[(L - 1) * np + 9], g_vecp[L - 1], g_o[L - 1], &g_xa_pre);
    epi_done = true;
  } else if (c.out_norm) {  // back through out_norm and the last layer's epilogue in one kernel
    Tensor g = at::empty_like(gX);
    const Tensor& on_w = P[P.size() - 2];
    check(tmdnet_ln_bwd_epilogue_w(dcode(gX), static_cast<int>(N), static_cast<int>(H), ptr(gX), ptr(A.x_pre),
                                   ptr(A.mean_o), ptr(A.rstd_o), ptr(on_w), nullptr, nullptr, ptr(g), ptr(gV),
                                   ptr(A.vecp[L - 1]), ptr(A.o[L - 1]), ptr(g_vecp[L - 1]), ptr(g_o[L - 1]), nullptr, 0,
                                   stream_of(gX)),
          "tmdnet_ln_bwd_epilogue_w");
    gX = g;
    epi_done = true;
  }
  for (int64_t l = L - 1; l >= 0; --l) {
    const Tensor* p = P.data() + l * np;
    if (!epi_done)
      check(tmdnet_et_epilogue_bwd_acc(dcode(gX), static_cast<int>(N), static_cast<int>(H), ptr(gX), ptr(gV),
                                       ptr(A.vecp[l]), ptr(A.o[l]), ptr(g_vecp[l]), ptr(g_o[l]), 0, stream_of(gX)),
            "tmdnet_et_epilogue_bwd_acc");
    Tensor g_xa = g_xa_pre;
    g_xa_pre = Tensor();
    if (!g_xa.defined()) {
      g_xa = at::empty({N, H}, o);
      gemm_into(g_o[l], p[9], false, Tensor(), g_xa, false);
    }
    const bool hv = A.vec[l].defined();
    Tensor g_vec_in = hv ? at::empty({N, 3, H}, o) : Tensor();
    Tensor g_qkv = at::empty({N, 5 * H}, o);
    Tensor dpk, dpv, pk, pv;
    if (has_e) {  // (distance_influence "none": no projection rows at all)
      Tensor pkv = A.batched ? A.pkv_all.narrow(1, l * D, D) : A.pkv_all;
      Tensor dpkv = A.batched ? dpkv_all.narrow(1, l * D, D) : Tensor();
      if (!A.batched) {
        dpkv = at::empty({E, D}, o);
        proj_into(dpkv_all, A.pk->dkv_w.narrow(0, l * D, D), Tensor(), Tensor(), dpkv);
        pkv = at::empty({E, D}, o);  // the forward's rows of this layer again (not kept for large graphs)
        proj_into(A.pkv_all, A.pk->dkv_w.narrow(0, l * D, D), Tensor(), A.pk->dkv_b.narrow(0, l * D, D), pkv);
      }
      if (c.hk) { pk = pkv.narrow(1, 0, H); dpk = dpkv.narrow(1, 0, H); }
      if (c.hv) { pv = pkv.narrow(1, H * int64_t(c.hk), 3 * H); dpv = dpkv.narrow(1, H * int64_t(c.hk), 3 * H); }
    }
    const Tensor& qkv = A.qkv[l];
    const int flags = TMDNET_ACC_VEC_RESIDUAL | (l < L - 1 ? TMDNET_ACC_EDGE : 0) | static_cast<int>(c.acts);
    Tensor gq = g_qkv.narrow(1, 0, H), gk = g_qkv.narrow(1, H, H), gv = g_qkv.narrow(1, 2 * H, 3 * H);
    const float* qb = static_cast<const float*>(qkv.data_ptr());
    check(tmdnet_et_message_bwd(dcode(gX), static_cast<int>(N), static_cast<int>(H), static_cast<int>(c.heads),
                                ptr<int32_t>(g.row_ptr), ptr<int32_t>(g.src), static_cast<int>(E), qb, ld(qkv),
                                qb + H, ld(qkv), qb + 2 * H, ld(qkv), ptr(A.vec[l]), ptr(pk), ld(pk),
                                ptr(pv), ld(pv), ptr(C), ptr(u), ptr(g_xa), ptr(gV), ptr(gq), ptr(gk), ptr(gv),
                                ptr(g_vec_in), nullptr, nullptr, ptr(g_C), ptr(g_u), has_e ? ptr(dpk) : nullptr,
                                has_e ? ptr(dpv) : nullptr, has_e ? ptr(g_r) : nullptr, flags, nullptr, nullptr,
                                stream_of(gX)),
          "tmdnet_et_message_bwd");
    Tensor g_xn = at::empty({N, H}, o);
    if (hv)
      gemm2_into(g_qkv, A.pk->qkv_w[l], false, g_xn, false, g_vecp[l].view({3 * N, 3 * H}), p[8], false,
                 g_vec_in.view({3 * N, H}), true);
    else
      gemm_into(g_qkv, A.pk->qkv_w[l], false, Tensor(), g_xn, false);
    const bool prev = l > 0;
    Tensor g_x;
    if (nf && prev) {
      g_x = lnbwd_oproj(g_xn, A.x[l], A.mean[l], A.rstd[l], p[0], gX, g_vec_in, A.vecp[l - 1], A.o[l - 1],
                        P[(l - 1) * np + 9], g_vecp[l - 1], g_o[l - 1], &g_xa_pre);
    } else {
      g_x = at::empty_like(g_xn);
      check(tmdnet_ln_bwd_epilogue_w(dcode(gX), static_cast<int>(N), static_cast<int>(H), ptr(g_xn), ptr(A.x[l]),
                                     ptr(A.mean[l]), ptr(A.rstd[l]), ptr(p[0]), ptr(gX), nullptr, ptr(g_x),
                                     ptr(g_vec_in), prev ? ptr(A.vecp[l - 1]) : nullptr,
                                     prev ? ptr(A.o[l - 1]) : nullptr, prev ? ptr(g_vecp[l - 1]) : nullptr,
                                     prev ? ptr(g_o[l - 1]) : nullptr, nullptr, 0, stream_of(gX)),
            "tmdnet_ln_bwd_epilogue_w");
    }
    epi_done = prev;
    gX = g_x;
    gV = g_vec_in;
  }
  return {gX, g_r, g_C, g_u};
}

struct StackIn {  // the operator's non-parameter tensors
  Tensor x, f, dist, C, u, mu, beta;
  G g;
};

// gradients of <(gX, gV), (x_out, vec_out)> w.r.t. (x, dist, C, u, params) by recompute; ``create`` keeps
// the graph (higher orders).  `want`: per leaf, whether its gradient is wanted.
variable_list stack_vjp(const StackIn& in, const std::vector<Tensor>& P, const StackCfg& c, const Tensor& gX,
                        const Tensor& gV, bool create) {
  at::AutoGradMode enable(true);
  variable_list leaves = {in.x.detach().requires_grad_(true), in.dist.detach().requires_grad_(true),
                          in.C.detach().requires_grad_(true), in.u.detach().requires_grad_(true)};
  std::vector<Tensor> Pl;
  for (const auto& t : P) Pl.push_back(t.detach().requires_grad_(true));
  auto out = stack_composite(leaves[0], leaves[1], leaves[2], leaves[3], in.mu, in.beta, Pl, in.g, c);
  variable_list all = leaves;
  all.insert(all.end(), Pl.begin(), Pl.end());
  return torch::autograd::grad({out.first, out.second}, all, {gX, gV}, create, create, true);
}

struct EtStackBwd : public Function<EtStackBwd> {
  // (gX, gV, x, dist, C, u, mu, beta, row_ptr, src, dst, params...) -> (g_x, g_dist, g_C, g_u, g_params...)
  static variable_list forward(AutogradContext* ctx, const Tensor& gX, const Tensor& gV, const Tensor& x,
                               const Tensor& dist, const Tensor& C, const Tensor& u, const Tensor& mu,
                               const Tensor& beta, const Tensor& row_ptr, const Tensor& src, const Tensor& dst,
                               c10::intrusive_ptr<StackActs> acts, StackCfg cfg, bool want_params,
                               at::TensorList params) {
    std::vector<Tensor> P(params.begin(), params.end());
    StackIn in{x, Tensor(), dist, C, u, mu, beta, G{row_ptr, src, dst, Tensor()}};
    variable_list res;
    if (!want_params) {
      res = stack_backward_dr(*acts, gX.contiguous(), gV.contiguous(), dist, C, u, mu, beta, P, in.g, cfg);
      // no parameter gradients: zero-size placeholders (a custom Function's outputs must be defined), made
      // without a fill -- at::zeros per parameter cost ~2 us of host time each, ~0.2 ms per C2 force pass
      const auto ox = opts(x);
      for (size_t i = 0; i < P.size(); ++i) res.push_back(at::empty({0}, ox));
    } else {  // training through TorchScript: autograd over the restatement
      at::NoGradGuard off;
      res = stack_vjp(in, P, cfg, gX, gV, false);
      // a parameter the restatement does not use (layer 0's vec_proj: vec = 0) gets a zero gradient,
      // as autograd over the reference's layer loop gives it
      for (size_t i = 0; i < P.size(); ++i)
        if (!res[4 + i].defined()) res[4 + i] = at::zeros_like(P[i]);
      for (auto& t : res)
        if (!t.defined()) t = at::zeros({0}, opts(x));
    }
    keep_cfg(ctx, cfg);
    keep_graph(ctx, in.g);
    variable_list sv = {gX, gV, x, dist, C, u, mu, beta};
    sv.insert(sv.end(), P.begin(), P.end());
    ctx->save_for_backward(sv);
    return res;
  }

  // the second order (force-matching training) and beyond: recompute the restatement, differentiate twice
  static variable_list backward(AutogradContext* ctx, variable_list ggs) {
    auto sv = ctx->get_saved_variables();
    const StackCfg c = cfg_of(ctx);
    G g = graph_of(ctx);
    const bool create = at::GradMode::is_enabled();
    at::AutoGradMode enable(true);
    variable_list leaves;
    for (size_t i = 0; i < sv.size(); ++i)
      leaves.push_back((i == 6 || i == 7) ? sv[i] : sv[i].detach().requires_grad_(true));  // mu, beta fixed
    std::vector<Tensor> P(leaves.begin() + 8, leaves.end());
    auto out = stack_composite(leaves[2], leaves[3], leaves[4], leaves[5], sv[6], sv[7], P, g, c);
    variable_list prim = {leaves[2], leaves[3], leaves[4], leaves[5]};
    prim.insert(prim.end(), P.begin(), P.end());
    auto first = torch::autograd::grad({out.first, out.second}, prim, {leaves[0], leaves[1]}, true, true, true);
    variable_list fs, fg;
    for (size_t i = 0; i < first.size() && i < ggs.size(); ++i)
      if (ggs[i].defined() && ggs[i].numel() && first[i].defined() && first[i].requires_grad()) {
        fs.push_back(first[i]);
        fg.push_back(ggs[i]);
      }
    // (gX, gV, x, dist, C, u, mu, beta, row_ptr, src, dst, acts, cfg, want_params, params...)
    variable_list res(14 + P.size());
    if (fs.empty()) return res;
    variable_list wrt = {leaves[0], leaves[1], leaves[2], leaves[3], leaves[4], leaves[5]};
    wrt.insert(wrt.end(), P.begin(), P.end());
    auto second = torch::autograd::grad(fs, wrt, fg, true, create, true);
    for (int i = 0; i < 6; ++i) res[i] = second[i];
    for (size_t i = 0; i < P.size(); ++i) res[14 + i] = second[6 + i];
    return res;
  }
};

// The stack's forward launches (EtStack::forward; also the fused inference operator et_energy_forces):
// returns (x_out, vec_out) and fills the intermediates A the dr-mode backward reads.
std::pair<Tensor, Tensor> stack_forward(const Tensor& x_in, const Tensor& f_in, const Tensor& dist, const Tensor& C_in,
                                        const Tensor& u_in, const Tensor& row_ptr, const Tensor& src,
                                        const Tensor& dst, const StackCfg& c, const std::vector<Tensor>& P,
                                        StackActs* A) {
    require_gpu(x_in, "et_stack");
    TORCH_CHECK(x_in.scalar_type() == at::kFloat, "et_stack: fp32 only (the model's per-layer loop serves fp64)");
    const int64_t np = stack_np(c.hk, c.hv);
    const int64_t nP = static_cast<int64_t>(P.size()) - (c.out_norm ? 2 : 0);
    TORCH_CHECK(nP > 0 && nP % np == 0, "et_stack: ", P.size(), " parameters for ", np, " per layer");
    const int64_t L = nP / np;
    Tensor x = x_in.contiguous(), f = f_in.contiguous(), C = C_in.contiguous(), u = u_in.contiguous();
    G g{row_ptr, src, dst, Tensor()};
    const int64_t N = x.size(0), H = x.size(1), E = g.E(), D = (int64_t(c.hk) + 3 * int64_t(c.hv)) * H;
    TORCH_CHECK(dist.size(0) == E && C.size(0) == E && u.size(0) == E && (!(c.hk || c.hv) || f.size(0) == E),
                "et_stack: per-edge shapes");
    auto o = opts(x);
    A->pk = pack_stack(P, L, np, c.hk, c.hv);
    const bool has_e = c.hk || c.hv;
    // every layer's projection rows in one GEMM unless that buffer would exceed 2 GB (large graphs:
    // per layer, recomputed by the backward)
    A->batched = E * L * D * 4 <= (int64_t(2) << 30);
    if (has_e) {
      if (A->batched) {
        A->pkv_all = at::empty({E, L * D}, o);
        proj_into(f, A->pk->dkv_w, A->pk->dkv_wp, A->pk->dkv_b, A->pkv_all);
      } else {
        A->pkv_all = f;
      }
    }
    auto epi_ln = [&](const Tensor& xx, const Tensor& vv, const Tensor& vp, const Tensor& oo, const Tensor& va,
                      const Tensor& w, const Tensor& b, Tensor* xo, Tensor* vo, Tensor* xn, Tensor* mean, Tensor* rstd) {
      *xn = at::empty({N, H}, o);
      *mean = at::empty({N, 1}, o);
      *rstd = at::empty({N, 1}, o);
      if (oo.defined()) {
        *xo = at::empty({N, H}, o);
        *vo = at::empty({N, 3, H}, o);
      }
      check(tmdnet_et_epilogue_ln_fwd(dcode(xx), static_cast<int>(N), static_cast<int>(H), ptr(xx), ptr(vv), ptr(vp),
                                      ptr(oo), ptr(va), ptr(w), ptr(b), kLnEps, oo.defined() ? ptr(*xo) : nullptr,
                                      oo.defined() ? ptr(*vo) : nullptr, ptr(*xn), ptr(*mean), ptr(*rstd),
                                      stream_of(xx)),
            "tmdnet_et_epilogue_ln_fwd");
    };
    Tensor vec, xn, mean, rstd, unused0, unused1;
    const bool nf = node_fuse_ok(N, H);
    if (!nf) epi_ln(x, Tensor(), Tensor(), Tensor(), Tensor(), P[0], P[1], &unused0, &unused1, &xn, &mean, &rstd);
    for (int64_t l = 0; l < L; ++l) {
      const Tensor* p = P.data() + l * np;
      Tensor qkv = at::empty({N, 5 * H}, o), vecp;
      if (nf) {  // LayerNorm + [q|k|v] + vec_proj in one launch
        ln_mix(x, p[0], p[1], A->pk->qkv_w[l], A->pk->qkv_b[l], vec, p[8], qkv, &vecp, &xn, &mean, &rstd);
      } else {
        gemm_into(xn, A->pk->qkv_w[l], true, A->pk->qkv_b[l], qkv, false);
        if (vec.defined()) {
          vecp = at::empty({N, 3, 3 * H}, o);
          gemm_into(vec.view({3 * N, H}), p[8], true, Tensor(), vecp.view({3 * N, 3 * H}), false);
        }
      }
      Tensor pkv, pk, pv;
      if (has_e) {
        if (A->batched) {
          pkv = A->pkv_all.narrow(1, l * D, D);
        } else {
          pkv = at::empty({E, D}, o);
          proj_into(f, A->pk->dkv_w.narrow(0, l * D, D), Tensor(), A->pk->dkv_b.narrow(0, l * D, D), pkv);
        }
        if (c.hk) pk = pkv.narrow(1, 0, H);
        if (c.hv) pv = pkv.narrow(1, H * int64_t(c.hk), 3 * H);
      }
      Tensor xa = at::empty({N, H}, o), veca = at::empty({N, 3, H}, o);
      float* qb = static_cast<float*>(qkv.data_ptr());
      check(tmdnet_et_message_fwd(dcode(x), static_cast<int>(N), static_cast<int>(H), static_cast<int>(c.heads),
                                  ptr<int32_t>(row_ptr), ptr<int32_t>(src), static_cast<int>(E), qb, ld(qkv), qb + H,
                                  ld(qkv), qb + 2 * H, ld(qkv), ptr(vec), ptr(pk), ld(pk), ptr(pv), ld(pv), ptr(C),
                                  ptr(u), ptr(xa), ptr(veca), static_cast<int>(c.acts), nullptr, nullptr,
                                  stream_of(x)),
            "tmdnet_et_message_fwd");
      Tensor oo = at::empty({N, 3 * H}, o);
      Tensor xo, vo;
      if (nf && l + 1 < L) {  // o_proj + the epilogue in one launch (the next LayerNorm: its mix)
        oproj_epi(xa, p[9], p[10], x, vec, vecp, veca, oo, &xo, &vo);
      } else {
        gemm_into(xa, p[9], true, p[10], oo, false);
      }
      A->x.push_back(x); A->vec.push_back(vec); A->xn.push_back(xn); A->mean.push_back(mean);
      A->rstd.push_back(rstd); A->qkv.push_back(qkv); A->vecp.push_back(vecp); A->xa.push_back(xa);
      A->o.push_back(oo);
      if (nf && l + 1 < L) {
        // (x_out, vec_out came with o; the next LayerNorm runs in the next layer's mix)
      } else if (l + 1 < L) {
        epi_ln(x, vec, vecp, oo, veca, P[(l + 1) * np], P[(l + 1) * np + 1], &xo, &vo, &xn, &mean, &rstd);
      } else if (c.out_norm) {  // the last epilogue + out_norm: x_out = LN(x_pre)
        epi_ln(x, vec, vecp, oo, veca, P[P.size() - 2], P[P.size() - 1], &xo, &vo, &xn, &mean, &rstd);
        A->x_pre = xo;
        A->mean_o = mean;
        A->rstd_o = rstd;
        xo = xn;
      } else {
        xo = at::empty({N, H}, o);
        vo = at::empty({N, 3, H}, o);
        check(tmdnet_et_epilogue_fwd(dcode(x), static_cast<int>(N), static_cast<int>(H), ptr(x), ptr(vec), ptr(vecp),
                                     ptr(oo), ptr(veca), ptr(xo), ptr(vo), stream_of(x)),
              "tmdnet_et_epilogue_fwd");
      }
      x = xo;
      vec = vo;
    }
  return {x, vec};
}

struct EtStack : public Function<EtStack> {
  static variable_list forward(AutogradContext* ctx, const Tensor& x_in, const Tensor& f_in, const Tensor& dist,
                               const Tensor& C_in, const Tensor& u_in, const Tensor& mu, const Tensor& beta,
                               const Tensor& row_ptr, const Tensor& src, const Tensor& dst, StackCfg c,
                               at::TensorList params) {
    std::vector<Tensor> P(params.begin(), params.end());
    auto A = c10::make_intrusive<StackActs>();
    auto xv = stack_forward(x_in, f_in, dist, C_in, u_in, row_ptr, src, dst, c, P, A.get());
    Tensor x = xv.first, vec = xv.second;
    G g{row_ptr, src, dst, Tensor()};
    ctx->saved_data["fwd_state"] = c10::IValue::make_capsule(A);  // the forward intermediates (StackActs)
    keep_cfg(ctx, c);
    keep_graph(ctx, g);
    variable_list sv = {x_in, dist, C_in, u_in, mu, beta};
    sv.insert(sv.end(), P.begin(), P.end());
    ctx->save_for_backward(sv);
    return {x, vec};
  }

  static variable_list backward(AutogradContext* ctx, variable_list go) {
    auto sv = ctx->get_saved_variables();
    const StackCfg c = cfg_of(ctx);
    G g = graph_of(ctx);
    auto A = c10::static_intrusive_pointer_cast<StackActs>(ctx->saved_data["fwd_state"].toCapsule());
    std::vector<Tensor> P(sv.begin() + 6, sv.end());
    // gradients: one per argument (x, f, dist, C, u, mu, beta, row_ptr, src, dst, cfg, params...);
    // needs_input_grad counts tensor arguments only (cfg has no edge): parameter i is edge 10 + i
    variable_list res(11 + P.size());
    bool want_params = false;
    for (size_t i = 0; i < P.size(); ++i) want_params = want_params || ctx->needs_input_grad(10 + i);
    const bool any = want_params || ctx->needs_input_grad(0) || ctx->needs_input_grad(2) ||
                     ctx->needs_input_grad(3) || ctx->needs_input_grad(4);
    if (!any) return res;
    Tensor x = sv[0];
    const int64_t N = x.size(0), H = x.size(1);
    Tensor gX = go[0].defined() ? go[0] : at::zeros({N, H}, opts(x));
    Tensor gV = go[1].defined() ? go[1] : at::zeros({N, 3, H}, opts(x));
    auto o = EtStackBwd::apply(gX, gV, x, sv[1], sv[2], sv[3], sv[4], sv[5], g.row_ptr, g.src, g.dst, A, c,
                               want_params, at::TensorList(P));  // (a TensorList: every parameter an input)
    auto sized = [](const Tensor& t) { return t.defined() && t.numel() ? t : Tensor(); };  // none / zero-size
    res[0] = sized(o[0]);
    res[2] = sized(o[1]);
    res[3] = sized(o[2]);
    res[4] = sized(o[3]);
    if (want_params)
      for (size_t i = 0; i < P.size(); ++i)
        if (ctx->needs_input_grad(10 + i) && o[4 + i].defined() && o[4 + i].numel()) res[11 + i] = o[4 + i];
    return res;
  }
};

std::tuple<Tensor, Tensor> et_stack(const Tensor& x, const Tensor& f, const Tensor& dist, const Tensor& cutoff,
                                    const Tensor& unit, const Tensor& mu, const Tensor& beta, const Tensor& row_ptr,
                                    const Tensor& src, const Tensor& dst, double cutoff_lower, double cutoff_upper,
                                    int64_t rbf_type, int64_t heads, bool has_dk, bool has_dv, bool out_norm,
                                    at::TensorList params, int64_t acts) {
  const c10::OptionalDeviceGuard guard(x.device());
  StackCfg c{heads, rbf_type, cutoff_lower, cutoff_upper, has_dk, has_dv, out_norm, acts};
  auto r = EtStack::apply(x, f, dist, cutoff, unit, mu.detach().to(dist.scalar_type()).contiguous(),
                          beta.detach().to(dist.scalar_type()).contiguous(), row_ptr, src, dst, c, params);
  return {r[0], r[1]};
}


// ----------------------------------------------------------------------------- large systems (C5 size)
// The eager path's large-system forms, for the fused inference operator: Morton renumbering of the atoms
// (kernels.spatial_permutation), pair-shared projection rows (tmdnet_pair_index), the planar v layout and
// the fused-projection layer kernels (et_fused.hip; et_stack FEP) -- no projection row of any layer is
// written: per layer only the split weight image (128 KB) and per evaluation the pair rows' RBF fragments.
// size switches (kernels.REORDER_MIN_ATOMS, et_stack.FEP_MIN_EDGES); tests force them on small systems
// through tmdnet::set_large_system_thresholds
static int64_t g_reorder_min_atoms = 16384, g_fep_min_edges = 131072;

std::vector<int64_t> set_large_system_thresholds(int64_t min_atoms, int64_t min_edges) {
  std::vector<int64_t> prev{g_reorder_min_atoms, g_fep_min_edges};
  if (min_atoms >= 0) g_reorder_min_atoms = min_atoms;
  if (min_edges >= 0) g_fep_min_edges = min_edges;
  return prev;
}

Tensor spread10(Tensor x) {
  x = at::bitwise_and(x, 0x3FF);
  x = at::bitwise_and(at::bitwise_or(x, at::bitwise_left_shift(x, 16)), 0x030000FF);
  x = at::bitwise_and(at::bitwise_or(x, at::bitwise_left_shift(x, 8)), 0x0300F00F);
  x = at::bitwise_and(at::bitwise_or(x, at::bitwise_left_shift(x, 4)), 0x030C30C3);
  return at::bitwise_and(at::bitwise_or(x, at::bitwise_left_shift(x, 2)), 0x09249249);
}

// molecule-major, then Morton order of cutoff-sized cells (kernels.spatial_permutation)
Tensor spatial_permutation(const Tensor& pos, const Tensor& batch, double cell, const Tensor& box, bool periodic) {
  Tensor p = pos.detach();
  if (periodic && box.defined() && box.numel() == 9) {
    Tensor b = box.detach().to(at::kCPU).to(at::kDouble).contiguous();
    const double* bd = b.data_ptr<double>();
    p = at::stack({at::remainder(p.select(1, 0), bd[0]), at::remainder(p.select(1, 1), bd[4]),
                   at::remainder(p.select(1, 2), bd[8])},
                  1);
  }
  Tensor lo = std::get<0>(p.min(0));
  Tensor c = at::clamp(((p - lo) / cell).to(at::kLong), 0, 1023);
  Tensor key = at::bitwise_or(at::bitwise_or(spread10(c.select(1, 0)), at::bitwise_left_shift(spread10(c.select(1, 1)), 1)),
                              at::bitwise_left_shift(spread10(c.select(1, 2)), 2));
  key = key + batch.to(at::kLong) * (int64_t(1) << 31);
  return at::argsort(key, /*stable=*/true);
}

// planar [x | v1 | v2] row j of v = row vperm[j] of the reference per-head interleave (et_stack._v_perm)
Tensor v_perm(int64_t H, int64_t heads, const Tensor& like) {
  const int64_t d = H / heads;
  Tensor j = at::arange(3 * H, like.options().dtype(at::kLong));
  Tensor part = at::floor_divide(j, H), rem = at::remainder(j, H);
  return at::floor_divide(rem, d) * (3 * d) + part * d + at::remainder(rem, d);
}

struct FusedAux {  // per evaluation: pair numbering + RBF fragments; per layer: planar weights + images
  Tensor pair_row, pair_edge, frags, dscale, qkv_perm;
  int64_t n_rows = 0;
  std::vector<Tensor> qkv_w, qkv_b, img, wsc, bias;
};

// the RBF fragments of the pair rows (tmdnet_fep_frags_f32), once per evaluation
void fused_frags(FusedAux* F, const Tensor& dist, const Tensor& mu, const Tensor& beta, double cl, double cu,
                 int64_t rbf, void* st) {
  if (F->frags.defined()) return;
  const int64_t R = mu.size(0);
  Tensor r_rows = dist.index_select(0, F->pair_edge.to(at::kLong)).contiguous();
  F->n_rows = r_rows.size(0);
  F->frags = at::empty({std::max<int64_t>(1, static_cast<int64_t>(tmdnet_fep_frags_bytes(F->n_rows, R) / 2))},
                       opts(dist).dtype(at::kHalf));
  F->dscale = at::empty({std::max<int64_t>(1, F->n_rows)}, opts(dist));
  check(tmdnet_fep_frags_f32(F->n_rows, static_cast<int>(R), ptr(r_rows), ptr(mu), ptr(beta), cl, cu,
                             static_cast<int>(rbf), ptr(F->frags), ptr(F->dscale), st),
        "tmdnet_fep_frags_f32");
}

// the fused-projection stack forward (et_stack._forward_layers with meta.fep): returns (x_out, vec_out)
std::pair<Tensor, Tensor> stack_forward_fused(const Tensor& x_in, const Tensor& dist, const Tensor& C, const Tensor& u,
                                              const Tensor& row_ptr, const Tensor& src, const Tensor& mu,
                                              const Tensor& beta, const StackCfg& c, const std::vector<Tensor>& P,
                                              StackActs* A, FusedAux* F) {
  const int64_t np = stack_np(c.hk, c.hv);
  const int64_t L = (static_cast<int64_t>(P.size()) - 2) / np;
  Tensor x = x_in.contiguous();
  const int64_t N = x.size(0), H = x.size(1), E = src.size(0), R = mu.size(0), D = 4 * H;
  auto o = opts(x);
  void* st = stream_of(x);
  A->pk = pack_stack(P, L, np, c.hk, c.hv);
  // RBF fragments of the pair rows, once for every layer (the fused neighbour embedding may have made them)
  fused_frags(F, dist, mu, beta, c.cl, c.cu, c.rbf, st);
  Tensor vp = v_perm(H, c.heads, x);
  F->qkv_perm = at::cat({at::arange(2 * H, vp.options()), 2 * H + vp});
  Tensor one = at::cat({at::arange(H, vp.options()), H + vp});  // [dk | dv] rows in the planar order
  auto epi_ln = [&](const Tensor& xx, const Tensor& vv, const Tensor& vpp, const Tensor& oo, const Tensor& va,
                    const Tensor& w, const Tensor& b, Tensor* xo, Tensor* vo, Tensor* xn, Tensor* mean, Tensor* rstd) {
    *xn = at::empty({N, H}, o);
    *mean = at::empty({N, 1}, o);
    *rstd = at::empty({N, 1}, o);
    if (oo.defined()) {
      *xo = at::empty({N, H}, o);
      *vo = at::empty({N, 3, H}, o);
    }
    check(tmdnet_et_epilogue_ln_fwd(TMDNET_F32, static_cast<int>(N), static_cast<int>(H), ptr(xx), ptr(vv), ptr(vpp),
                                    ptr(oo), ptr(va), ptr(w), ptr(b), kLnEps, oo.defined() ? ptr(*xo) : nullptr,
                                    oo.defined() ? ptr(*vo) : nullptr, ptr(*xn), ptr(*mean), ptr(*rstd), st),
          "tmdnet_et_epilogue_ln_fwd");
  };
  Tensor vec, xn, mean, rstd, unused0, unused1;
  const bool nf = node_fuse_ok(N, H);
  if (!nf) epi_ln(x, Tensor(), Tensor(), Tensor(), Tensor(), P[0], P[1], &unused0, &unused1, &xn, &mean, &rstd);
  for (int64_t l = 0; l < L; ++l) {
    const Tensor* p = P.data() + l * np;
    F->qkv_w.push_back(A->pk->qkv_w[l].index_select(0, F->qkv_perm).contiguous());
    F->qkv_b.push_back(A->pk->qkv_b[l].index_select(0, F->qkv_perm).contiguous());
    const Tensor W = A->pk->dkv_w.narrow(0, l * D, D).index_select(0, one).contiguous();
    const Tensor Wb = A->pk->dkv_b.narrow(0, l * D, D).index_select(0, one).contiguous();
    F->img.push_back(at::empty({static_cast<int64_t>(tmdnet_fep_image_bytes(static_cast<int>(D), static_cast<int>(R)) / 2)},
                               o.dtype(at::kHalf)));
    F->wsc.push_back(at::empty({D}, o));
    F->bias.push_back(at::empty({D}, o));
    check(tmdnet_fep_split_f32(static_cast<int>(D), static_cast<int>(R), ptr(W), static_cast<int>(R), ptr(Wb),
                               ptr(F->img[l]), ptr(F->wsc[l]), ptr(F->bias[l]), st),
          "tmdnet_fep_split_f32");
    Tensor qkv = at::empty({N, 5 * H}, o), vecp;
    if (nf) {
      ln_mix(x, p[0], p[1], F->qkv_w[l], F->qkv_b[l], vec, p[8], qkv, &vecp, &xn, &mean, &rstd);
    } else {
      gemm_into(xn, F->qkv_w[l], true, F->qkv_b[l], qkv, false);
      if (vec.defined()) {
        vecp = at::empty({N, 3, 3 * H}, o);
        gemm_into(vec.view({3 * N, H}), p[8], true, Tensor(), vecp.view({3 * N, 3 * H}), false);
      }
    }
    Tensor xa = at::empty({N, H}, o), veca = at::empty({N, 3, H}, o);
    const float* qb = static_cast<const float*>(qkv.data_ptr());
    check(tmdnet_et_fused_fwd_f32(static_cast<int>(N), static_cast<int>(H), static_cast<int>(c.heads), static_cast<int>(R),
                                  ptr<int32_t>(row_ptr), ptr<int32_t>(src), static_cast<int>(E), qb, ld(qkv), qb + H,
                                  ld(qkv), qb + 2 * H, ld(qkv), ptr(vec), ptr(C), ptr(u), ptr<int32_t>(F->pair_row),
                                  ptr(F->frags), F->n_rows, ptr(F->img[l]), ptr(F->wsc[l]), ptr(F->bias[l]), ptr(xa),
                                  ptr(veca), TMDNET_ET_V_PLANAR, st),
          "tmdnet_et_fused_fwd_f32");
    Tensor oo = at::empty({N, 3 * H}, o);
    Tensor xo, vo;
    if (nf && l + 1 < L)
      oproj_epi(xa, p[9], p[10], x, vec, vecp, veca, oo, &xo, &vo);
    else
      gemm_into(xa, p[9], true, p[10], oo, false);
    A->x.push_back(x); A->vec.push_back(vec); A->xn.push_back(xn); A->mean.push_back(mean);
    A->rstd.push_back(rstd); A->qkv.push_back(qkv); A->vecp.push_back(vecp); A->xa.push_back(xa);
    A->o.push_back(oo);
    if (nf && l + 1 < L) {
      // (x_out, vec_out came with o; the next LayerNorm runs in the next layer's mix)
    } else if (l + 1 < L) {
      epi_ln(x, vec, vecp, oo, veca, P[(l + 1) * np], P[(l + 1) * np + 1], &xo, &vo, &xn, &mean, &rstd);
    } else {  // the last epilogue + out_norm
      epi_ln(x, vec, vecp, oo, veca, P[P.size() - 2], P[P.size() - 1], &xo, &vo, &xn, &mean, &rstd);
      A->x_pre = xo;
      A->mean_o = mean;
      A->rstd_o = rstd;
      xo = xn;
    }
    x = xo;
    vec = vo;
  }
  return {x, vec};
}

// its force-pass backward (et_stack._backward_layers, dr mode, fused): (g_x, g_r, g_C, g_u)
variable_list stack_backward_fused(const StackActs& A, const FusedAux& F, Tensor gX, Tensor gV, const Tensor& C,
                                   const Tensor& u, const Tensor& row_ptr, const Tensor& src, const std::vector<Tensor>& P,
                                   const StackCfg& c, int64_t R) {
  const int64_t N = gX.size(0), H = gX.size(1), E = src.size(0), np = stack_np(c.hk, c.hv);
  const int64_t L = static_cast<int64_t>(A.x.size());
  auto o = opts(gX);
  void* st = stream_of(gX);
  Tensor g_C = at::empty({E}, o), g_u = at::empty({E, 3}, o), g_r = at::empty({E}, o);
  const size_t wsb = tmdnet_et_fused_bwd_workspace_bytes(static_cast<int>(E));
  Tensor ws = wsb ? at::empty({static_cast<int64_t>(wsb / 4)}, o) : Tensor();
  std::vector<Tensor> g_o(L), g_vecp(L);
  for (int64_t l = 0; l < L; ++l) {
    g_o[l] = at::empty({N, 3 * H}, o);
    if (A.vec[l].defined()) g_vecp[l] = at::empty({N, 3, 3 * H}, o);
  }
  const bool nf = node_fuse_ok(N, H);
  Tensor g_xa_pre;
  if (nf) {
    gX = lnbwd_oproj(gX, A.x_pre, A.mean_o, A.rstd_o, P[P.size() - 2], Tensor(), gV, A.vecp[L - 1], A.o[L - 1],
                     P[(L - 1) * np + 9], g_vecp[L - 1], g_o[L - 1], &g_xa_pre);
  } else {  // back through out_norm and the last layer's epilogue in one kernel
    Tensor g = at::empty_like(gX);
    check(tmdnet_ln_bwd_epilogue_w(TMDNET_F32, static_cast<int>(N), static_cast<int>(H), ptr(gX), ptr(A.x_pre),
                                   ptr(A.mean_o), ptr(A.rstd_o), ptr(P[P.size() - 2]), nullptr, nullptr, ptr(g), ptr(gV),
                                   ptr(A.vecp[L - 1]), ptr(A.o[L - 1]), ptr(g_vecp[L - 1]), ptr(g_o[L - 1]), nullptr, 0,
                                   st),
          "tmdnet_ln_bwd_epilogue_w");
    gX = g;
  }
  for (int64_t l = L - 1; l >= 0; --l) {
    const Tensor* p = P.data() + l * np;
    Tensor g_xa = g_xa_pre;
    g_xa_pre = Tensor();
    if (!g_xa.defined()) {
      g_xa = at::empty({N, H}, o);
      gemm_into(g_o[l], p[9], false, Tensor(), g_xa, false);
    }
    const bool hv = A.vec[l].defined();
    Tensor g_vec_in = hv ? at::empty({N, 3, H}, o) : Tensor();
    Tensor g_qkv = at::empty({N, 5 * H}, o);
    const Tensor& qkv = A.qkv[l];
    const float* qb = static_cast<const float*>(qkv.data_ptr());
    float* gb = static_cast<float*>(g_qkv.data_ptr());
    const int flags = TMDNET_ACC_VEC_RESIDUAL | (l < L - 1 ? TMDNET_ACC_EDGE : 0) | TMDNET_ET_V_PLANAR;
    check(tmdnet_et_fused_bwd_f32(static_cast<int>(N), static_cast<int>(H), static_cast<int>(c.heads), static_cast<int>(R),
                                  ptr<int32_t>(row_ptr), ptr<int32_t>(src), static_cast<int>(E), qb, ld(qkv), qb + H,
                                  ld(qkv), qb + 2 * H, ld(qkv), ptr(A.vec[l]), ptr(C), ptr(u), ptr<int32_t>(F.pair_row),
                                  ptr(F.frags), ptr(F.dscale), F.n_rows, ptr(F.img[l]), ptr(F.wsc[l]), ptr(F.bias[l]),
                                  ptr(g_xa), ptr(gV), gb, gb + H, gb + 2 * H, ptr(g_vec_in), ptr(g_C), ptr(g_u), ptr(g_r),
                                  flags, ptr(ws), wsb, st),
          "tmdnet_et_fused_bwd_f32");
    Tensor g_xn = at::empty({N, H}, o);
    if (hv)
      gemm2_into(g_qkv, F.qkv_w[l], false, g_xn, false, g_vecp[l].view({3 * N, 3 * H}), p[8], false,
                 g_vec_in.view({3 * N, H}), true);
    else
      gemm_into(g_qkv, F.qkv_w[l], false, Tensor(), g_xn, false);
    const bool prev = l > 0;
    Tensor g_x;
    if (nf && prev) {
      g_x = lnbwd_oproj(g_xn, A.x[l], A.mean[l], A.rstd[l], p[0], gX, g_vec_in, A.vecp[l - 1], A.o[l - 1],
                        P[(l - 1) * np + 9], g_vecp[l - 1], g_o[l - 1], &g_xa_pre);
    } else {
      g_x = at::empty_like(g_xn);
      check(tmdnet_ln_bwd_epilogue_w(TMDNET_F32, static_cast<int>(N), static_cast<int>(H), ptr(g_xn), ptr(A.x[l]),
                                     ptr(A.mean[l]), ptr(A.rstd[l]), ptr(p[0]), ptr(gX), nullptr, ptr(g_x), ptr(g_vec_in),
                                     prev ? ptr(A.vecp[l - 1]) : nullptr, prev ? ptr(A.o[l - 1]) : nullptr,
                                     prev ? ptr(g_vecp[l - 1]) : nullptr, prev ? ptr(g_o[l - 1]) : nullptr, nullptr, 0,
                                     st),
            "tmdnet_ln_bwd_epilogue_w");
    }
    gX = g_x;
    gV = g_vec_in;
  }
  return {gX, g_r, g_C, g_u};
}

// ----------------------------------------------------------------------------- fused inference
// A whole ET energy + force evaluation (TorchMD_Net.forward with derivative=True, reference
// models/model.py:232-300, torchmd_et.py:154-187, output_modules.py:80-115) as ONE operator with no autograd
// graph: the launches of the eager graph-replayed path issued from C++ -- embeddings, neighbour list, edge
// geometry, neighbour embedding, the fused layer stack, the EquivariantScalar head with its per-atom
// Jacobian, the per-molecule sum, then the force pass (the head's Jacobian scaled by -std, the stack's dr-mode
// backward, the neighbour-embedding / geometry / neighbour backward passes, every second consumer's
// gradient summed in-kernel).  For TorchScript inference (MD engines, reference README.md:6): the
// scripted model takes it in eval mode; its outputs carry no autograd graph.
std::tuple<Tensor, Tensor> et_energy_forces(
    const Tensor& z_arg, const Tensor& pos_in, const Tensor& batch_arg, const Tensor& box, bool use_periodic, double cl,
    double cu, int64_t max_pairs, bool loop, const std::string& strategy, bool check_errors, const Tensor& emb_w,
    const c10::optional<Tensor>& nb_emb_w_, const c10::optional<Tensor>& nb_dist_w_,
    const c10::optional<Tensor>& nb_dist_b_, const c10::optional<Tensor>& nb_comb_w_,
    const c10::optional<Tensor>& nb_comb_b_, const Tensor& mu_in, const Tensor& beta_in, int64_t rbf_type,
    int64_t heads, bool has_dk, bool has_dv, bool out_norm, at::TensorList stack_params, int64_t acts,
    at::TensorList head_params, const Tensor& std_in, const Tensor& mean_in) {
  const c10::OptionalDeviceGuard guard(pos_in.device());
  require_gpu(pos_in, "et_energy_forces");
  TORCH_CHECK(pos_in.scalar_type() == at::kFloat && emb_w.scalar_type() == at::kFloat,
              "et_energy_forces: fp32 models only");
  TORCH_CHECK(head_params.size() == 12, "et_energy_forces: the EquivariantScalar head's 12 tensors");
  at::NoGradGuard ng;
  Tensor pos = pos_in.detach().contiguous(), z = z_arg, batch = batch_arg.contiguous();
  const int64_t N = z.size(0), H = emb_w.size(1), R = mu_in.size(0);
  // large systems: the spatially coherent atom numbering of the eager path (TorchMD_ET.forward); the
  // forces are returned in the caller's order
  Tensor perm;
  if (N >= g_reorder_min_atoms) {
    perm = spatial_permutation(pos, batch, cu, box, use_periodic);
    z = z.index_select(0, perm);
    pos = pos.index_select(0, perm).contiguous();
    batch = batch.index_select(0, perm).contiguous();
  }
  auto o = opts(pos);
  void* st = stream_of(pos);
  const int dt = TMDNET_F32;
  const Tensor mu = mu_in.detach().to(at::kFloat).contiguous(), beta = beta_in.detach().to(at::kFloat).contiguous();
  const Tensor zl = z.to(at::kLong).contiguous();
  // embeddings: both tables in one launch
  const Tensor nb_emb_w = val(nb_emb_w_);
  const bool nb = nb_emb_w.defined();
  Tensor x = at::empty({N, H}, o), xe = nb ? at::empty({N, H}, o) : Tensor();
  {
    const void* tabs[2] = {emb_w.data_ptr(), nb ? nb_emb_w.data_ptr() : nullptr};
    const int lts[2] = {static_cast<int>(emb_w.stride(0)), nb ? static_cast<int>(nb_emb_w.stride(0)) : 0};
    void* outs[2] = {x.data_ptr(), nb ? xe.data_ptr() : nullptr};
    const int lds[2] = {static_cast<int>(H), static_cast<int>(H)};
    check(tmdnet_embedding_fwd_f32(static_cast<int>(N), static_cast<int>(H), static_cast<int>(emb_w.size(0)),
                                   zl.data_ptr<int64_t>(), nb ? 2 : 1, tabs, lts, outs, lds, st),
          "tmdnet_embedding_fwd_f32");
  }
  // neighbour list (reference OptimizedDistance: resize_to_fit, check_errors)
  Tensor bx = box;
  if (strategy == "cell" && !use_periodic) {
    bx = at::zeros({3, 3}, at::TensorOptions().dtype(at::kDouble));
    bx[0][0] = 3.0 * cu;
    bx[1][1] = 3.0 * cu;
    bx[2][2] = 3.0 * cu;
  }
  Built B = nl_build(strategy, pos, batch, bx, use_periodic, cl, cu, max_pairs, loop, true, true, true);
  const int64_t found = B.num.item<int>();
  TORCH_CHECK(!check_errors || found <= max_pairs, "Found num_pairs(", found, ") > max_num_pairs(", max_pairs, ")");
  TORCH_CHECK(found <= max_pairs, "et_energy_forces: the force pass needs the full symmetric neighbour list");
  const int64_t E = found;
  const Tensor src = B.nb[0].narrow(0, 0, E), dst = B.nb[1].narrow(0, 0, E), tr = B.tr.narrow(0, 0, E);
  const Tensor dl = B.dl.narrow(0, 0, E), dist = B.dist.narrow(0, 0, E);
  const Tensor& row_ptr = B.row_ptr;
  // the fused-projection layer kernels (et_stack FEP: C5-size graphs, the configuration they implement)
  const bool fused = E >= g_fep_min_edges && H == 128 && heads == 8 && (R == 32 || R == 64) && has_dk && has_dv &&
                     acts == 0 && out_norm;
  FusedAux F;
  if (fused) {  // pair numbering: both directions of a pair read one fragment row
    F.pair_row = at::empty({E}, iopts(pos));
    F.pair_edge = at::empty({(E + N) / 2}, iopts(pos));
    Tensor pws = at::empty({static_cast<int64_t>(std::max<size_t>(16, tmdnet_pair_index_workspace_bytes(static_cast<int>(N))))},
                           pos.options().dtype(at::kByte));
    const bool sorted_rows = strategy != "cell";  // brute / shared rows list sources ascending
    check(tmdnet_pair_index(static_cast<int>(N), ptr<int32_t>(row_ptr), ptr<int32_t>(src), ptr<int32_t>(dst),
                            ptr<int32_t>(tr), static_cast<int>(E), ptr<int32_t>(B.num), sorted_rows ? 1 : 0,
                            ptr<int32_t>(F.pair_row), ptr<int32_t>(F.pair_edge), static_cast<int>(F.pair_edge.size(0)),
                            pws.data_ptr(), static_cast<size_t>(pws.numel()), st),
          "tmdnet_pair_index");
  }
  // edge geometry
  Tensor f = at::empty({E, R}, o), C = at::empty({E}, o), u = at::empty({E, 3}, o);
  check(tmdnet_edge_geom_fwd(dt, static_cast<int>(E), static_cast<int>(R), static_cast<int>(rbf_type),
                             ptr<int32_t>(src), ptr<int32_t>(dst), ptr(dl), ptr(dist), ptr(mu), ptr(beta), cl, cu,
                             ptr(f), ptr(C), ptr(u), st),
        "tmdnet_edge_geom_fwd");
  // neighbour embedding: W = distance_proj(f); [x | x_nb] by the aggregation kernel; combine.  Large systems
  // (the fused stack's envelope): distance_proj formed inside the aggregation kernel from the pair rows'
  // fragments (tmdnet_nbr_fused_fwd_f32, eager kernels.nbr_embed_fused) -- no E x H rows
  Tensor W, cat, x1 = x, nimg, nwsc, nbias;
  const bool nb_fused = nb && fused;
  if (nb) {
    cat = at::empty({N, 2 * H}, o);
    float* cb = static_cast<float*>(cat.data_ptr());
    if (nb_fused) {
      fused_frags(&F, dist, mu, beta, cl, cu, rbf_type, st);
      const Tensor dw = val(nb_dist_w_).contiguous(), db = val(nb_dist_b_).contiguous();
      nimg = at::empty({static_cast<int64_t>(tmdnet_fep_image_bytes(static_cast<int>(H), static_cast<int>(R)) / 2)},
                       o.dtype(at::kHalf));
      nwsc = at::empty({H}, o);
      nbias = at::empty({H}, o);
      check(tmdnet_fep_split_f32(static_cast<int>(H), static_cast<int>(R), ptr(dw), static_cast<int>(dw.stride(0)),
                                 ptr(db), ptr(nimg), ptr(nwsc), ptr(nbias), st),
            "tmdnet_fep_split_f32");
      check(tmdnet_nbr_fused_fwd_f32(static_cast<int>(N), static_cast<int>(H), static_cast<int>(R),
                                     ptr<int32_t>(row_ptr), ptr<int32_t>(src), static_cast<int>(E), ptr(xe),
                                     static_cast<int>(H), ptr(C), ptr<int32_t>(F.pair_row), ptr(F.frags), F.n_rows,
                                     ptr(nimg), ptr(nwsc), ptr(nbias), cb + H, static_cast<int>(2 * H), ptr(x), cb, st),
            "tmdnet_nbr_fused_fwd_f32");
    } else {
      W = at::empty({E, H}, o);
      gemm_into(f, val(nb_dist_w_), true, val(nb_dist_b_), W, false);
      check(tmdnet_nbr_embed_fwd(dt, static_cast<int>(N), static_cast<int>(H), ptr<int32_t>(row_ptr),
                                 ptr<int32_t>(src), static_cast<int>(E), ptr(xe), static_cast<int>(H), ptr(W),
                                 static_cast<int>(H), ptr(C), cb + H, static_cast<int>(2 * H), ptr(x), cb, st),
            "tmdnet_nbr_embed_fwd");
    }
    x1 = at::empty({N, H}, o);
    gemm_into(cat, val(nb_comb_w_), true, val(nb_comb_b_), x1, false);
  }
  // the layer stack
  StackCfg c{heads, rbf_type, cl, cu, has_dk, has_dv, out_norm, acts};
  std::vector<Tensor> P(stack_params.begin(), stack_params.end());
  StackActs A;
  auto xv = fused ? stack_forward_fused(x1, dist, C, u, row_ptr, src, mu, beta, c, P, &A, &F)
                  : stack_forward(x1, f, dist, C, u, row_ptr, src, dst, c, P, &A);
  const Tensor xo = xv.first.contiguous(), vo = xv.second.contiguous();
  // the head (+ per-atom Jacobian) and the per-molecule sum
  Tensor y_atom = at::empty({N, 1}, o), jx = at::empty({N, H}, o), jv = at::empty({N, 3, H}, o);
  const void* hw[12];
  for (int i = 0; i < 12; ++i) hw[i] = head_params[i].data_ptr();
  // the MFMA head over 16-atom tiles (eager kernels._eq_head_x3) when its envelope holds and the system is
  // past the per-atom kernel's crossover (kernels.HEAD_X3_MIN_ATOMS), else per atom
  bool head_x3 = dt == TMDNET_F32 && N >= 768 && tmdnet_eq_head_x3_pieces_bytes(static_cast<int>(H)) > 0;
  for (int i : {3, 5, 9}) head_x3 = head_x3 && (reinterpret_cast<uintptr_t>(hw[i]) & 15) == 0;
  for (int i = 0; i < 12; ++i) head_x3 = head_x3 && head_params[i].is_contiguous();
  if (head_x3) {
    const size_t pb = tmdnet_eq_head_x3_pieces_bytes(static_cast<int>(H));
    Tensor pieces = at::empty({static_cast<int64_t>(pb / 2)}, o.dtype(at::kShort));
    check(tmdnet_eq_head_x3_split_f32(static_cast<int>(H), hw, pieces.data_ptr(), st), "tmdnet_eq_head_x3_split_f32");
    const int64_t O = H / 2;
    const int64_t nk[10][2] = {{H + O, H}, {H, 2 * H}, {H, H}, {O, O}, {O, 2 * O},
                               {2 * O, O}, {O, O},     {H, H}, {2 * H, H}, {H, H + O}};
    const void* pc[10];
    const int16_t* base = static_cast<const int16_t*>(pieces.data_ptr());
    int64_t off = 0;
    for (int i = 0; i < 10; ++i) {
      pc[i] = base + off;
      off += 3 * nk[i][0] * nk[i][1];
    }
    const void* hv[5] = {hw[3], hw[5], hw[9], hw[10], hw[11]};
    check(tmdnet_eq_head_x3_f32(static_cast<int>(N), static_cast<int>(H), ptr(xo), ptr(vo), pc, hv, ptr(y_atom),
                                ptr(jx), ptr(jv), nullptr, st),
          "tmdnet_eq_head_x3_f32");
  } else {
    check(tmdnet_eq_head_fwd(dt, static_cast<int>(N), static_cast<int>(H), ptr(xo), ptr(vo), hw, ptr(y_atom), ptr(jx),
                             ptr(jv), st),
          "tmdnet_eq_head_fwd");
  }
  const int64_t n_mol = batch.max().item<int64_t>() + 1;  // (the reference reduce's dim_size, a host read)
  const Tensor sd = std_in.to(at::kFloat).contiguous(), mn = mean_in.to(at::kFloat).contiguous();
  Tensor y = at::empty({n_mol, 1}, o);
  check(tmdnet_atom_sum_fwd(dt, static_cast<int>(N), static_cast<int>(n_mol), ptr(y_atom), batch.data_ptr<int64_t>(),
                            ptr(sd), ptr(mn), ptr(y), st),
        "tmdnet_atom_sum_fwd");
  // force pass, seeded with -1 (neg_dy directly)
  Tensor seed = at::full({n_mol, 1}, -1.0, o), g_atom = at::empty({N, 1}, o);
  check(tmdnet_atom_sum_bwd(dt, static_cast<int>(N), static_cast<int>(n_mol), ptr(seed), batch.data_ptr<int64_t>(),
                            ptr(sd), ptr(g_atom), st),
        "tmdnet_atom_sum_bwd");
  Tensor gX = at::empty({N, H}, o), gV = at::empty({N, 3, H}, o);
  check(tmdnet_eq_head_bwd(dt, static_cast<int>(N), static_cast<int>(H), ptr(g_atom), ptr(jx), ptr(jv), ptr(gX),
                           ptr(gV), st),
        "tmdnet_eq_head_bwd");
  G g{row_ptr, src, dst, tr};
  auto gs = fused ? stack_backward_fused(A, F, gX, gV, C, u, row_ptr, src, P, c, R)
                  : stack_backward_dr(A, gX, gV, dist, C, u, mu, beta, P, g, c);  // (g_x1, g_r, g_C, g_u)
  Tensor gf, gC_nb;
  if (nb_fused) {  // dr mode: g_C and g_r per edge, added to the stack's (no E x H / E x R gradient rows)
    Tensor g_cat = at::empty({N, 2 * H}, o);
    gemm_into(gs[0], val(nb_comb_w_), false, Tensor(), g_cat, false);
    const float* gcb = static_cast<const float*>(g_cat.data_ptr());
    check(tmdnet_nbr_fused_bwd_f32(static_cast<int>(N), static_cast<int>(H), static_cast<int>(R), ptr<int32_t>(row_ptr),
                                   ptr<int32_t>(src), static_cast<int>(E), ptr(xe), static_cast<int>(H), ptr(C),
                                   ptr<int32_t>(F.pair_row), ptr(F.frags), ptr(F.dscale), F.n_rows, ptr(nimg),
                                   ptr(nwsc), ptr(nbias), gcb + H, static_cast<int>(2 * H), ptr(gs[2]), ptr(gs[1]),
                                   TMDNET_ACC_EDGE, st),
          "tmdnet_nbr_fused_bwd_f32");
  } else if (nb) {
    Tensor g_cat = at::empty({N, 2 * H}, o);
    gemm_into(gs[0], val(nb_comb_w_), false, Tensor(), g_cat, false);
    Tensor gW = at::empty({E, H}, o);
    gC_nb = at::empty({E}, o);
    const float* gcb = static_cast<const float*>(g_cat.data_ptr());
    check(tmdnet_nbr_embed_bwd(dt, static_cast<int>(N), static_cast<int>(H), ptr<int32_t>(row_ptr), ptr<int32_t>(src),
                               static_cast<int>(E), ptr(xe), static_cast<int>(H), ptr(W), static_cast<int>(H), ptr(C),
                               gcb + H, static_cast<int>(2 * H), nullptr, ptr(gW), ptr(gC_nb), st),
          "tmdnet_nbr_embed_bwd");
    gf = at::empty({E, R}, o);
    gemm_into(gW, val(nb_dist_w_), false, Tensor(), gf, false);
  }
  Tensor g_r = at::empty({E}, o), g_dl = at::empty({E, 3}, o);
  check(tmdnet_edge_geom_bwd_multi(dt, static_cast<int>(E), static_cast<int>(R), static_cast<int>(rbf_type),
                                   ptr<int32_t>(src), ptr<int32_t>(dst), ptr(dl), ptr(dist), ptr(mu), ptr(beta), cl, cu,
                                   ptr(gf), nullptr, nullptr, ptr(gs[2]), ptr(gC_nb), nullptr, ptr(gs[3]), ptr(g_r),
                                   ptr(g_dl), st),
        "tmdnet_edge_geom_bwd_multi");
  Tensor neg_dy = at::empty({N, 3}, o);
  check(tmdnet_nl_backward_multi(dt, static_cast<int>(N), ptr<int32_t>(row_ptr), ptr<int32_t>(tr), static_cast<int>(E),
                                 ptr(g_dl), ptr(g_r), ptr(gs[1]), ptr(dl), ptr(dist), ptr(neg_dy), st),
        "tmdnet_nl_backward_multi");
  if (perm.defined()) {  // back to the caller's atom order
    Tensor out = at::empty_like(neg_dy);
    out.index_copy_(0, perm, neg_dy);
    neg_dy = out;
  }
  return {y, neg_dy};
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
        "Tensor row_ptr, Tensor src, Tensor dst, int heads, int acts=0) -> (Tensor x, Tensor vec)");
  m.def("tn_embed(Tensor P, Tensor Q, Tensor W, Tensor cutoff, Tensor unit, Tensor row_ptr, Tensor src, "
        "Tensor dst, float self0_mult) -> Tensor");
  m.def("tn_message(Tensor edge_attr, Tensor comp, Tensor row_ptr, Tensor src, Tensor dst, float self0_mult) -> "
        "Tensor");
  m.def("et_stack(Tensor x, Tensor f, Tensor dist, Tensor cutoff, Tensor unit, Tensor mu, Tensor beta, "
        "Tensor row_ptr, Tensor src, Tensor dst, float cutoff_lower, float cutoff_upper, int rbf_type, int heads, "
        "bool has_dk, bool has_dv, bool out_norm, Tensor[] params, int acts=0) -> (Tensor x, Tensor vec)");
  // (no-op: et_stack forms its stacked weights on every call; kept for callers of the cached form)
  m.def("et_stack_invalidate() -> ()", tmdt::et_stack_invalidate);
  // the large-system switches of et_energy_forces (Morton renumbering from min_atoms atoms, the fused
  // projection kernels from min_edges edges; < 0 keeps a value); returns the previous values
  m.def("set_large_system_thresholds(int min_atoms, int min_edges) -> int[]", tmdt::set_large_system_thresholds);
  m.def("et_energy_forces(Tensor z, Tensor pos, Tensor batch, Tensor box, bool use_periodic, float cutoff_lower, "
        "float cutoff_upper, int max_pairs, bool loop, str strategy, bool check_errors, Tensor emb_w, "
        "Tensor? nb_emb_w, Tensor? nb_dist_w, Tensor? nb_dist_b, Tensor? nb_comb_w, Tensor? nb_comb_b, Tensor mu, "
        "Tensor beta, int rbf_type, int heads, bool has_dk, bool has_dv, bool out_norm, Tensor[] stack_params, "
        "int acts, Tensor[] head_params, Tensor std, Tensor mean) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(tmdnet, CompositeImplicitAutograd, m) {
  m.impl("neighbor_graph", tmdt::neighbor_graph);
  m.impl("edge_geometry", tmdt::edge_geometry);
  m.impl("nbr_embed", tmdt::nbr_embed);
  m.impl("et_message", tmdt::et_message);
  m.impl("tn_embed", tmdt::tn_embed);
  m.impl("tn_message", tmdt::tn_message);
  m.impl("et_stack", tmdt::et_stack);
  m.impl("et_energy_forces", tmdt::et_energy_forces);
}
