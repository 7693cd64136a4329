/* tmdnet.h -- C ABI of the MI355X-native TorchMD-NET hot path (libtmdnet_hip.so, gfx950).
 *
 * Plain pointers, sizes and an opaque hipStream_t (passed as void*); no torch types, no C++
 * exceptions across the boundary.  Every entry point returns 0 (TMDNET_OK) or a status code and
 * only ENQUEUES work on `stream` (no host synchronisation, no allocation: callers pass workspaces),
 * so every call is HIP-graph capturable.
 *
 * Device buffers are row-major and contiguous unless a leading dimension (ld*) is given.
 * `dtype` selects the floating type of every floating buffer of the call (TMDNET_F32/F64).
 * Edge lists are destination-grouped CSR:  row t = edges e in [row_ptr[t], row_ptr[t+1]) whose
 * destination (reference edge_index[1]) is t; src[e] (reference edge_index[0]) is its source.
 * Indices at or beyond `max_pairs` are ignored (capacity overflow, reference common.cuh:106-116).
 */
#ifndef TMDNET_H
#define TMDNET_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { TMDNET_OK = 0, TMDNET_BAD_ARGUMENT = 1, TMDNET_UNSUPPORTED = 2, TMDNET_LAUNCH_FAILED = 3,
       TMDNET_WORKSPACE_TOO_SMALL = 4 };
enum { TMDNET_F32 = 0, TMDNET_F64 = 1 };
enum { TMDNET_NL_BRUTE = 0, TMDNET_NL_SHARED = 1, TMDNET_NL_CELL = 2 };
enum { TMDNET_RBF_EXPNORM = 0, TMDNET_RBF_GAUSS = 1 };
enum { TMDNET_ACC_VEC_RESIDUAL = 1, TMDNET_ACC_EDGE = 2 };
/* tmdnet_et_message_bwd accumulate bit: ADD the node gradients (gq, gk, gv, gvec_in) and the edge
 * gradients (gpk, gpv) to the output buffers' contents (the second order injects its cotangents there
 * first) instead of overwriting them. */
enum { TMDNET_ACC_GRADS = 32 };
/* v / pv row layout flag of the ET message entry points: planar rows [x | v1 | v2] of H channels each
 * instead of the reference's per-head interleave [h][x|v1|v2] of d channels (torchmd_et.py:282-291).
 * Planar rows make every 16-byte-per-lane load of a row segment contiguous (measured 4-7 % on the C5
 * forward).  Gradients of v / pv are written in the same layout. */
enum { TMDNET_ET_V_PLANAR = 4 };
/* tmdnet_et_message_bwd2_ex flags: accumulate d_cut / d_unit (ACC_EDGE) and d_grad_vec (ACC_GVEC)
 * into the caller's buffers instead of overwriting them. */
enum { TMDNET_BWD2_ACC_EDGE = 8, TMDNET_BWD2_ACC_GVEC = 16 };
/* tmdnet_et_message_bwd accumulate bit: the dr-mode backward as the two passes (destination, then
 * source) instead of the merged pass that serves both roles of a node from one read of each pair row
 * (the default from 16384 nodes; same results up to summation order). */
enum { TMDNET_ET_TWO_PASS = 64 };
/* Activations of the ET message entry points (tmdnet_et_message_fwd flags, _bwd accumulate, _bwd2 /
 * _bwd2_ex flags): bits 8-11 = the dk / dv projections' activation (reference EquivariantMultiHeadAttention
 * `activation`, torchmd_et.py:285-291), bits 12-15 = the attention activation (`attn_activation`,
 * torchmd_et.py:316), coded as the reference act_class_mapping (models/utils.py:579-584): SiLU (0, the
 * default), ShiftedSoftplus, Tanh, Sigmoid.  Other codes: TMDNET_BAD_ARGUMENT.  (The fused-projection
 * entry points tmdnet_et_fused_* implement SiLU only.) */
enum { TMDNET_ACT_SILU = 0, TMDNET_ACT_SSP = 1, TMDNET_ACT_TANH = 2, TMDNET_ACT_SIGMOID = 3 };
#define TMDNET_ET_ACT(kv, attn) (((kv) << 8) | ((attn) << 12))

/* ------------------------------------------------------------------------------------------
 * Neighbour list.  Replaces torchmdnet_neighbors::get_neighbor_pairs
 *   (reference torchmdnet/neighbors/neighbors.cpp:3-5; CUDA forward_brute/_shared/_cell,
 *    neighbors_cuda_brute.cuh:269-309, neighbors_cuda_shared.cuh:71-106,
 *    neighbors_cuda_cell.cuh:338-378; output contract common.cuh:64-116).
 * Outputs (reference layout): neighbors int32 [2][max_pairs] (row 0 = source, row 1 = destination),
 * deltas [max_pairs][3] (= pos[src]-pos[dst], minimum image), distances [max_pairs],
 * num_pairs int32[1] = number of pairs FOUND (may exceed max_pairs; extra pairs are dropped).
 * pad_output=1 fills unused slots with -1 / 0 exactly like the reference; 0 leaves them untouched.
 * row_ptr (int32[n_atoms+1], nullable) receives the CSR offsets (not clamped to max_pairs).
 * transpose_map (int32[max_pairs], nullable) receives T[e] = index of the reversed edge (or -1);
 * only meaningful when include_transpose=1.
 * box9: row-major 3x3 box vectors on the HOST (reduced triclinic form), may be NULL if not periodic.
 * The cell strategy needs a diagonal box (the caller supplies 3*cutoff when not periodic, as
 * reference utils.py:199-202 does).
 */
size_t tmdnet_nl_workspace_bytes(int n_atoms, int strategy, const double* box9, double cutoff_upper);
int tmdnet_nl_build(int dtype, int strategy, const void* pos, const int64_t* batch, int n_atoms,
                    const double* box9, int use_periodic, double cutoff_lower, double cutoff_upper,
                    int max_pairs, int loop, int include_transpose, int32_t* neighbors, void* deltas,
                    void* distances, int32_t* num_pairs, int32_t* row_ptr, int32_t* transpose_map,
                    int pad_output, void* workspace, size_t workspace_bytes, void* stream);
/* tmdnet_nl_build plus the pair numbering of tmdnet_pair_index in the same launches (sorted rows:
 * brute / shared strategies, include_transpose with a transpose_map): pair_row [max_pairs] and
 * pair_edge [n_pair_slots] as tmdnet_pair_index fills them, with no extra launch (the canonical
 * counts ride on the count pass, their scan on the row scan, the numbers on the transpose pass).
 * The cell strategy returns TMDNET_BAD_ARGUMENT here (use tmdnet_pair_index). */
int tmdnet_nl_build_paired(int dtype, int strategy, const void* pos, const int64_t* batch, int n_atoms,
                           const double* box9, int use_periodic, double cutoff_lower, double cutoff_upper,
                           int max_pairs, int loop, int include_transpose, int32_t* neighbors, void* deltas,
                           void* distances, int32_t* num_pairs, int32_t* row_ptr, int32_t* transpose_map,
                           int pad_output, void* workspace, size_t workspace_bytes, int32_t* pair_row,
                           int32_t* pair_edge, int n_pair_slots, void* stream);

/* Backward of the neighbour op w.r.t. positions (reference NeighborAutograd::backward,
 * neighbors_cuda.cu:43-71) as a segmented CSR reduction (no atomics, deterministic):
 *   g[e] = r[e]==0 ? 0 : gdelta[e] + delta[e]/r[e]*gr[e];  dpos[n] = sum_{e in row n} g[T[e]] - g[e].
 * Requires a symmetric list (include_transpose=1) and its transpose_map.  grad_deltas or
 * grad_distances may be NULL (treated as zero).  grad_pos [n_atoms][3] is overwritten. */
int tmdnet_nl_backward(int dtype, int n_atoms, const int32_t* row_ptr, const int32_t* transpose_map,
                       int max_pairs, const void* grad_deltas, const void* grad_distances,
                       const void* deltas, const void* distances, void* grad_pos, void* stream);
/* The same with a second distance gradient (NULL allowed) summed in: the distances' second consumer
 * (the ET layer stack's force-pass g_r beside the edge geometry's), no separate add launch. */
int tmdnet_nl_backward_multi(int dtype, int n_atoms, const int32_t* row_ptr, const int32_t* transpose_map,
                             int max_pairs, const void* grad_deltas, const void* grad_distances,
                             const void* grad_distances2, const void* deltas, const void* distances,
                             void* grad_pos, void* stream);

/* The same backward for ANY list the op returns (half lists with include_transpose=0, capacity-
 * truncated lists, padding slots -1): one lane per slot of neighbors [2][max_pairs], g scattered to
 * both ends with atomics, exactly the reference's index_add_ pair (neighbors_cuda.cu:58-68; so,
 * like it, the fp summation order is not fixed).  grad_pos [n_atoms][3] is zeroed, then
 * accumulated.  Used by the raw torchmdnet_neighbors::get_neighbor_pairs op (libtmdnet_torch.so). */
int tmdnet_nl_backward_edges(int dtype, int n_atoms, const int32_t* neighbors, int max_pairs,
                             const void* grad_deltas, const void* grad_distances, const void* deltas,
                             const void* distances, void* grad_pos, void* stream);

/* Second order of tmdnet_nl_backward (the double backward the reference gets by differentiating
 * NeighborAutograd::backward's index_add pair, neighbors_cuda.cu:43-71).  gg_pos [n][3] is the
 * cotangent of grad_pos.  Per edge e = (src -> dst) with w = gg[src]-gg[dst], u = delta/r:
 *   d_grad_deltas[e] = w,  d_grad_distances[e] = u.w  (0 when r == 0),
 *   d_pos[n] = sum_{e in row n} h[T[e]] - h[e],  h[e] = grad_distances[e]/r (w - u (u.w)).
 * grad_distances NULL = zero (d_pos = 0).  d_grad_deltas / d_grad_distances may be NULL (not
 * computed); when given, all max_pairs rows are written (padding slots 0).  Same list
 * requirements as tmdnet_nl_backward. */
int tmdnet_nl_backward2(int dtype, int n_atoms, const int32_t* row_ptr, const int32_t* src,
                        const int32_t* transpose_map, int max_pairs, const void* grad_distances,
                        const void* deltas, const void* distances, const void* gg_pos, void* d_pos,
                        void* d_grad_deltas, void* d_grad_distances, void* stream);

/* ------------------------------------------------------------------------------------------
 * Edge geometry: radial basis + cosine cutoff + unit vectors, fused.  Replaces
 *   ExpNormalSmearing.forward / GaussianSmearing.forward (reference models/utils.py:339-344,
 *   298-300), CosineCutoff.forward (utils.py:368-390), and the d_ij normalisation of
 *   TorchMD_ET.forward (torchmd_et.py:173-174) / TensorNet.forward (tensornet.py:223-226).
 * rbf_type EXPNORM: f[e][k] = C0(r) exp(-beta_k (exp(alpha (cl - r)) - mu_k)^2), C0 = cosine
 *   cutoff (0, cu), alpha = 5/(cu-cl);  GAUSS: f[e][k] = exp(coeff * (r - mu_k)^2) (coeff = beta_0).
 * C[e] = CosineCutoff(cl, cu)(r);  unit[e] = self edge (src==dst) ? delta : delta / |delta|.
 * Any output pointer may be NULL (not computed). */
int tmdnet_edge_geom_fwd(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src,
                         const int32_t* dst, const void* deltas, const void* dist, const void* mu,
                         const void* beta, double cutoff_lower, double cutoff_upper, void* rbf,
                         void* cutoff, void* unit, void* stream);
/* tmdnet_edge_geom_fwd plus the RBF features of the edges rows[p] into rbf_rows [n_rows][num_rbf]
 * in the same launch (the ET layer stack's pair rows: replaces a gather of rbf). */
int tmdnet_edge_geom_fwd_rows(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src,
                              const int32_t* dst, const void* deltas, const void* dist, const void* mu,
                              const void* beta, double cutoff_lower, double cutoff_upper, void* rbf,
                              void* cutoff, void* unit, const int32_t* rows, int n_rows, void* rbf_rows,
                              void* stream);
/* tmdnet_edge_geom_fwd_rows plus d rbf / d r of the same rows into drbf_rows [n_rows][num_rbf] (the ET
 * force pass's dr-mode operand, formed with the features; replaces a tmdnet_rbf_deriv launch). */
int tmdnet_edge_geom_fwd_rows2(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src,
                               const int32_t* dst, const void* deltas, const void* dist, const void* mu,
                               const void* beta, double cutoff_lower, double cutoff_upper, void* rbf,
                               void* cutoff, void* unit, const int32_t* rows, int n_rows, void* rbf_rows,
                               void* drbf_rows, void* stream);
/* Backward: given grad_rbf [E][R], grad_cutoff [E], grad_unit [E][3] (each nullable) produce
 * grad_dist [E] and grad_deltas [E][3] (both overwritten). */
/* Second order of tmdnet_edge_geom_bwd (force-matching training; replaces autograd's double
 * differentiation of reference utils.py:303-390 and the d_ij normalisation, torchmd_et.py:173-174):
 * the VJP of (grad_deltas, grad_dist) for their cotangents gg_deltas [E][3], gg_dist [E] (NULL = 0),
 * with respect to grad_rbf, grad_cutoff, grad_unit, dist, deltas (outputs; NULL = not wanted):
 *   d_grad_rbf[e][k] = gg_dist f_k'(r)   d_grad_cutoff = gg_dist C'(r)
 *   d_dist = gg_dist (sum_k grad_rbf_k f_k''(r) + grad_cutoff C''(r))
 *   d_grad_unit, d_deltas: the unit vector's Jacobian and its derivative (self edges: identity, 0). */
int tmdnet_edge_geom_bwd2(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src,
                          const int32_t* dst, const void* deltas, const void* dist, const void* mu,
                          const void* beta, double cutoff_lower, double cutoff_upper,
                          const void* grad_rbf, const void* grad_cutoff, const void* grad_unit,
                          const void* gg_deltas, const void* gg_dist, void* d_grad_rbf,
                          void* d_grad_cutoff, void* d_grad_unit, void* d_dist, void* d_deltas,
                          void* stream);
/* d rbf_k / d r of edges rows[p] (rows NULL: edge p), out [n_rows][R] -- the RBF derivative the ET
 * force pass contracts with the dk/dv projection (tmdnet_et_message_bwd's dpk / dpv rows). */
int tmdnet_rbf_deriv(int dtype, int num_rbf, int rbf_type, const void* dist, const void* mu,
                     const void* beta, double cutoff_lower, double cutoff_upper, const int32_t* rows,
                     int n_rows, void* out, void* stream);
int tmdnet_edge_geom_bwd(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src,
                         const int32_t* dst, const void* deltas, const void* dist, const void* mu,
                         const void* beta, double cutoff_lower, double cutoff_upper,
                         const void* grad_rbf, const void* grad_cutoff, const void* grad_unit,
                         void* grad_dist, void* grad_deltas, void* stream);
/* The same with up to three incoming gradients per rbf / cutoff output (one per consumer of that output,
 * summed in slot order in the kernel; NULL slots skipped) -- replaces the autograd engine's add launches
 * for outputs read by several modules (TensorNet's embedding and interaction layers, tensornet.py:222-230). */
int tmdnet_edge_geom_bwd_multi(int dtype, int n_edges, int num_rbf, int rbf_type, const int32_t* src,
                               const int32_t* dst, const void* deltas, const void* dist, const void* mu,
                               const void* beta, double cutoff_lower, double cutoff_upper, const void* grad_rbf,
                               const void* grad_rbf2, const void* grad_rbf3, const void* grad_cutoff,
                               const void* grad_cutoff2, const void* grad_cutoff3, const void* grad_unit,
                               void* grad_dist, void* grad_deltas, void* stream);

/* ------------------------------------------------------------------------------------------
 * Equivariant-Transformer edge message + aggregation (reference
 *   EquivariantMultiHeadAttention.message/aggregate, models/torchmd_et.py:314-347, with the SiLU of
 *   the dk/dv projections, torchmd_et.py:282-291, folded in).  For every edge e (s=src, t=dst),
 *   head h, channel c of the head (d = H/heads):
 *     a[e,h]   = silu( sum_c q[t,h,c] k[s,h,c] silu(pk[e,h,c]) ) * C[e]
 *     x[t,h,c]       += v[s,h,c] silu(pv[e,h,c]) a[e,h]
 *     vec[t,a,h,c]   += vec_in[s,a,h,c] v[s,h,d+c] silu(pv[e,h,d+c]) + v[s,h,2d+c] silu(pv[e,h,2d+c]) unit[e,a]
 *   q,k: [N][H] (ld_q, ld_k); v: [N][3H] head-interleaved [x|v1|v2] (ld_v); vec_in, vec: [N][3][H];
 *   pk: [E][H] (ld_pk), pv: [E][3H] (ld_pv): PRE-activation dk/dv projections (NULL = factor 1, i.e.
 *   distance_influence without keys / values).  x: [N][H].  `order` (nullable) permutes the
 *   destinations processed (locality only; results identical).  `pk_rows` (nullable): edge e reads
 *   its projection from pk / pv row pk_rows[e] instead of row e -- dk/dv depend on |r| only, so the
 *   two directions of a pair share one row (tmdnet_pair_index) and the projection GEMM runs over
 *   (E + N) / 2 rows instead of E.  Gradient outputs (gpk / gpv of the backward) stay per edge.
 * One wave64 per destination; outputs written once; no atomics; deterministic.
 */
int tmdnet_et_message_fwd(int dtype, int n_nodes, int hidden, int heads, const int32_t* row_ptr,
                          const int32_t* src, int max_pairs, const void* q, int ld_q, const void* k,
                          int ld_k, const void* v, int ld_v, const void* vec_in, const void* pk,
                          int ld_pk, const void* pv, int ld_pv, const void* cutoff, const void* unit,
                          void* x_out, void* vec_out, int flags, const int32_t* pk_rows,
                          const int32_t* order, void* stream);
/* Size switches of the message backward's launch forms (run-time tuning; tests force the large-graph
 * forms onto small graphs).  BOTH_MAX_NODES: below it the destination and source passes share one grid
 * (default 16384, env TMDNET_ET_FUSE); MERGED_MIN_NODES: from it the dr-mode force pass runs both roles in
 * one pass over the rows (default 16384, env TMDNET_ET_MERGED_MIN).  Returns the previous value (-1:
 * unknown key).  Not thread-safe against concurrent launches. */
#define TMDNET_TUNE_ET_BOTH_MAX_NODES 1
#define TMDNET_TUNE_ET_MERGED_MIN_NODES 2
int tmdnet_set_tuning(int key, int value);

/* Backward (two CSR passes, no atomics): destination pass -> gq, gpk, gpv, gcut, gunit; source
 * pass -> gk, gv, gvec_in.
 * PRECONDITION (source pass, and the merged dr-mode pass used for >= 16384 nodes): the edge list is
 * symmetric and pair-symmetric in its per-edge inputs -- for every edge e = (t <- s) the list holds
 * rev(e) = (s <- t) with cutoff[rev(e)] == cutoff[e], unit[rev(e)] == -unit[e] and the same projection
 * (pk / pv row, or pk_rows[rev(e)] == pk_rows[e]).  The source role of node s reads those values from
 * s's OWN row (edge e' = (s <- m)) as the reversed edge m <- s, so a list violating this gives wrong
 * gk / gv / gvec_in silently.  Every list the model builds satisfies it (dk, dv, cutoff depend on |r|
 * only; minimum-image deltas flip sign).  Checked on the device by the Python launcher when
 * TMDNET_LIB=debug or TMDNET_CHECK_SYMMETRY=1 (kernels.check_pair_symmetry).
 * Gradients are written with the leading dimension of the matching input (gq: ld_q, gk: ld_k,
 * gv: ld_v, gpk: ld_pk, gpv: ld_pv), so they can land directly in fused [q|k|v] / [dk|dv]
 * gradient buffers; gpk/gpv are gradients of the PRE-activation projections.
 * vec_in may be NULL (vec == 0, the first layer): its terms vanish and gvec_in is not written
 * (gvec_in may also be NULL).  accumulate (TMDNET_ACC_* bits): VEC_RESIDUAL -> gvec_in =
 * grad_vec + message part (the layer's identity residual); EDGE -> gcut/gunit are accumulated
 * (+=) instead of overwritten (one buffer shared by all layers).  Other buffers: overwritten; rows
 * [row_ptr[n_nodes], max_pairs) of gpk / gpv (static-capacity padding) are set to zero, and so are those rows of gcut / gunit. */
int tmdnet_et_message_bwd(int dtype, int n_nodes, int hidden, int heads, const int32_t* row_ptr,
                          const int32_t* src, int max_pairs, const void* q, int ld_q, const void* k,
                          int ld_k, const void* v, int ld_v, const void* vec_in, const void* pk,
                          int ld_pk, const void* pv, int ld_pv, const void* cutoff, const void* unit,
                          const void* grad_x, const void* grad_vec, void* gq, void* gk, void* gv,
                          void* gvec_in, void* gpk, void* gpv, void* gcut, void* gunit,
                          const void* dpk, const void* dpv, void* gdist, int accumulate,
                          const int32_t* pk_rows, const int32_t* order,
                          void* stream);  /* accumulate may also carry TMDNET_ET_V_PLANAR */
/* "dr mode" of the backward (gdist non-NULL; with TMDNET_ACC_EDGE it accumulates, without it overwrites): instead of storing gpk / gpv
 * (then normally NULL), the projection gradient of every edge is contracted in-kernel with dpk = d pk / d r
 * (dpk / dpv rows are read with ld_pk / ld_pv),
 * dpv = d pv / d r (rows and layout of pk / pv, read through pk_rows) and accumulated into
 * gdist[e] -- the force pass then needs neither the E x 4H gradient nor its GEMM.  gpk / gpv non-NULL
 * in dr mode: the projection gradient is stored as well (the recorded force pass of force-matching
 * training keeps it for its second order). */

/* Second-order backward: the VJP of tmdnet_et_message_bwd (forces differentiated again, reference
 * model.py:286-298 with create_graph=True).  gg_* are the cotangents of that call's outputs (gq, gk,
 * gv, gvec_in, gpk, gpv, gcut, gunit; all required, dense, zeros where unused; gg_q/gg_k [N][H],
 * gg_v [N][3H], gg_vec [N][3][H], gg_pk/gg_pv with leading dimensions).  Outputs: d_grad_x, d_grad_vec,
 * d_q, d_k [N][H], d_v [N][3H], d_vec [N][3][H] (d_k, d_v, d_vec accumulated with atomics: zero them
 * first; d_vec may be NULL when vec_in is NULL), d_pk [E][H], d_pv [E][3H], d_cut [E], d_unit [E][3]
 * (every row written, static-capacity padding rows [row_ptr[n_nodes], max_pairs) with zeros). */
int tmdnet_et_message_bwd2(int dtype, int n_nodes, int hidden, int heads, const int32_t* row_ptr,
                           const int32_t* src, int max_pairs, const void* q, int ld_q, const void* k,
                           int ld_k, const void* v, int ld_v, const void* vec_in, const void* pk,
                           int ld_pk, const void* pv, int ld_pv, const void* cutoff, const void* unit,
                           const void* grad_x, const void* grad_vec, const void* gg_q, const void* gg_k,
                           const void* gg_v, const void* gg_vec, const void* gg_pk, int ld_ggpk,
                           const void* gg_pv, int ld_ggpv, const void* gg_cut, const void* gg_unit,
                           void* d_grad_x, void* d_grad_vec, void* d_q, void* d_k, void* d_v,
                           void* d_vec, void* d_pk, void* d_pv, void* d_cut, void* d_unit, int flags,
                           void* stream);
/* tmdnet_et_message_bwd2 with row strides for the node cotangents / outputs (0 = dense) -- so the
 * cotangents can be column blocks of one [N][5H] buffer and d_q | d_k | d_v written into one -- and
 * a DETERMINISTIC source pass: with transpose (the reversed-edge map of tmdnet_nl_build) and
 * edge_scratch ([max_pairs][7][hidden] elements, 16-byte aligned) the source-node terms of every edge
 * are stored as a scratch row and summed per node over the reversed edges by a second kernel (no
 * atomics; d_k, d_v, d_vec are overwritten, no zero fill needed).  transpose / edge_scratch NULL:
 * atomics as tmdnet_et_message_bwd2.  pk_rows (nullable, as in tmdnet_et_message_fwd): edge e's
 * projection rows pk / pv are rows pk_rows[e] (pair-shared rows; gg_pk / gg_pv and d_pk / d_pv stay
 * per edge).  gg_pkv_scale (nullable, needs pk_rows): gg_pk / gg_pv are pair rows too, edge e's
 * cotangent being row pk_rows[e] scaled by gg_pkv_scale[e] (the force-matching second order: the
 * cotangent of the dr-mode g_r times d(dk,dv)/dr).  flags: TMDNET_ET_V_PLANAR | TMDNET_BWD2_ACC_*. */
int tmdnet_et_message_bwd2_ex(
    int dtype, int n_nodes, int hidden, int heads, const int32_t* row_ptr, const int32_t* src,
    const int32_t* transpose, int max_pairs, const void* q, int ld_q, const void* k, int ld_k,
    const void* v, int ld_v, const void* vec_in, const void* pk, int ld_pk, const void* pv, int ld_pv,
    const void* cutoff, const void* unit, const void* grad_x, const void* grad_vec, const void* gg_q,
    int ld_ggq, const void* gg_k, int ld_ggk, const void* gg_v, int ld_ggv, const void* gg_vec,
    const void* gg_pk, int ld_ggpk, const void* gg_pv, int ld_ggpv, const void* gg_cut,
    const void* gg_unit, void* d_grad_x, void* d_grad_vec, void* d_q, int ld_dq, void* d_k, int ld_dk,
    void* d_v, int ld_dv, void* d_vec, void* d_pk, int ld_dpk, void* d_pv, int ld_dpv, void* d_cut,
    void* d_unit, void* edge_scratch, const int32_t* pk_rows, const void* gg_pkv_scale, int flags,
    void* stream);

/* ET layer epilogue (reference torchmd_et.py:278-280, 309-311 + residuals 181-184), fused:
 *   vecp = vec_proj(vec) [N][3][3H] = [v1|v2|v3], o = o_proj(x_agg) [N][3H] = [o1|o2|o3]
 *   x_out = x + (sum_a v1*v2) * o2 + o3;  vec_out = vec + v3 * o1 + vec_agg.
 * vec and vecp may be NULL (vec == 0). */
int tmdnet_et_epilogue_fwd(int dtype, int n_nodes, int hidden, const void* x, const void* vec,
                           const void* vecp, const void* o, const void* vec_agg, void* x_out,
                           void* vec_out, void* stream);
/* Backward of the epilogue: grad_vecp [N][3][3H], grad_o [N][3H] (x, vec, vec_agg pass through). */
int tmdnet_et_epilogue_bwd(int dtype, int n_nodes, int hidden, const void* grad_x,
                           const void* grad_vec, const void* vecp, const void* o, void* grad_vecp,
                           void* grad_o, void* stream);
/* tmdnet_et_epilogue_bwd with accumulate != 0: grad_vecp / grad_o are ADDED to (they hold the cotangents
 * the force-loss second order injects; et_stack._backward_layers). */
int tmdnet_et_epilogue_bwd_acc(int dtype, int n_nodes, int hidden, const void* grad_x, const void* grad_vec,
                               const void* vecp, const void* o, void* grad_vecp, void* grad_o,
                               int accumulate, void* stream);

/* Epilogue of layer l fused with the LayerNorm of layer l+1 (torchmd_et.py:262; biased variance,
 * rstd = 1/sqrt(var + eps), as torch.native_layer_norm).  o == NULL: LayerNorm only (of x; x_out,
 * vec_out unused).  ln_w == NULL: epilogue only.  xn [N][H], mean [N], rstd [N]. */
int tmdnet_et_epilogue_ln_fwd(int dtype, int n_nodes, int hidden, const void* x, const void* vec,
                              const void* vecp, const void* o, const void* vec_agg, const void* ln_w,
                              const void* ln_b, double eps, void* x_out, void* vec_out, void* xn,
                              void* mean, void* rstd, void* stream);
/* grad_x = grad_res + LayerNorm backward of grad_xn (input x, saved mean / rstd, weight ln_w; no
 * weight gradients; grad_res NULL: no residual, e.g. the model's final out_norm); when o != NULL, then the epilogue backward of the previous layer with
 * (grad_x, grad_vec, vecp, o) -> grad_vecp, grad_o (as tmdnet_et_epilogue_bwd; vecp NULL = first
 * layer). */
int tmdnet_ln_bwd_epilogue(int dtype, int n_nodes, int hidden, const void* grad_xn, const void* x,
                           const void* mean, const void* rstd, const void* ln_w, const void* grad_res,
                           void* grad_x, const void* grad_vec, const void* vecp, const void* o,
                           void* grad_vecp, void* grad_o, void* stream);
/* tmdnet_ln_bwd_epilogue that also writes w_rows [N][H] = grad_xn * xhat, the per-row terms of the
 * LayerNorm weight gradient (its column sum; the bias gradient is the column sum of grad_xn), so a
 * training backward keeps the fused kernel and forms every layer's weight gradients in one batched
 * reduction (et_stack._backward_layers). */
int tmdnet_ln_bwd_epilogue_w(int dtype, int n_nodes, int hidden, const void* grad_xn, const void* x,
                             const void* mean, const void* rstd, const void* ln_w, const void* grad_res,
                             const void* grad_res2, void* grad_x, const void* grad_vec, const void* vecp,
                             const void* o, void* grad_vecp, void* grad_o, void* w_rows, int accumulate,
                             void* stream);
/* (grad_res2: a second residual term, NULL = none; accumulate != 0: grad_vecp / grad_o are ADDED to.) */

/* The ET layer's node mixes with the epilogue / LayerNorm pass folded in (et_nodemix.hip; fp32, hidden %
 * 64 == 0, hidden <= 256, 16-byte aligned x_agg / o_w).  Replaces tmdnet_gemm_f32(o_proj) +
 * tmdnet_et_epilogue_ln_fwd (reference torchmd_et.py:181-184, 278-280, 309-311): o [N][3H] = x_agg o_w^T +
 * o_b, then x_out, vec_out as tmdnet_et_epilogue_fwd (vecp NULL: first layer, vec unused).  o, x_out and
 * vec_out are bit-identical to the two-launch form. */
int tmdnet_et_oproj_epilogue_f32(int n_nodes, int hidden, const void* x_agg, const void* o_w, const void* o_b,
                                 const void* x, const void* vec, const void* vecp, const void* vec_agg, void* o,
                                 void* x_out, void* vec_out, void* stream);
/* LayerNorm(x) (affine, biased variance, rstd = 1/sqrt(var + eps); torchmd_et.py:262) -> xn [N][H], mean
 * [N], rstd [N], and out [N][n_out] = xn w^T + b (the [q|k|v] Linear, torchmd_et.py:264-266) -- with, when
 * vec != NULL, vec_out [3N][n_vec_out] = vec [3N][H] vec_w^T (vec_proj, torchmd_et.py:268) in the same
 * launch.  Replaces the LayerNorm half of tmdnet_et_epilogue_ln_fwd + tmdnet_gemm_f32([q|k|v], vec_proj).
 * fp32, hidden % 64 == 0, hidden <= 256, 16-byte aligned operands. */
int tmdnet_et_ln_mix_f32(int n_nodes, int hidden, const void* x, const void* ln_w, const void* ln_b, double eps,
                         const void* w, const void* b, int n_out, void* out, void* xn, void* mean, void* rstd,
                         const void* vec, const void* vec_w, int n_vec_out, void* vec_out, void* stream);
/* The force pass's mirror (et_nodemix.hip; fp32, hidden == 128): the LayerNorm backward of layer l
 * (tmdnet_ln_bwd_epilogue with grad_res, no weight rows) -> grad_x, the epilogue backward of layer l-1 ->
 * grad_vecp, grad_o (vecp NULL: layer l-1 is the first, grad_vecp unused), and grad_xa [N][H] = grad_o o_w
 * (o_w = layer l-1's o_proj weight [3H][H], torchmd_et.py:311) in one launch.  Replaces
 * tmdnet_ln_bwd_epilogue + tmdnet_gemm_f32(o_proj^T). */
int tmdnet_et_lnbwd_oproj_f32(int n_nodes, int hidden, const void* grad_xn, const void* x, const void* mean,
                              const void* rstd, const void* ln_w, const void* grad_res, const void* grad_vec,
                              const void* vecp, const void* o, const void* o_w, void* grad_x, void* grad_vecp,
                              void* grad_o, void* grad_xa, void* stream);

/* Second order of the layer tail (force-matching training, et_stack._second_order): layer l's
 * epilogue-backward VJP fused with layer l+1's LayerNorm-backward VJP, one wave per node.
 * Epilogue part (o != NULL): cotangents gb_o [N][3H], gb_vecp [N][3][3H] of tmdnet_et_epilogue_bwd's
 * outputs at (grad_x, grad_vec, vecp, o) -> gbar_x_out = gbar_x_in + its grad_x cotangent,
 * gbar_vec_out = gbar_vec_in (NULL = 0) + its grad_vec cotangent, vecp_bar, o_bar (the primal
 * cotangents); vecp NULL (first layer): only gb_o's third block reaches gbar_x_out.
 * LayerNorm part (ln_w != NULL): the VJP of g_x = LNB(grad_xn, x) (tmdnet_ln_bwd_epilogue without
 * residual) for the cotangent gbar_x_out (o NULL: gbar_x_in) -> gbar_grad_xn, x_bar, and the per-row
 * products w_bar_rows [N][H] whose column sum is ln_w's cotangent.  mean / rstd as saved by the
 * forward.  Every output written (no accumulation besides the *_in terms). */
int tmdnet_et_adjoint_epi_ln(int dtype, int n_nodes, int hidden, const void* gb_o, const void* gb_vecp,
                             const void* grad_x, const void* grad_vec, const void* vecp, const void* o,
                             const void* gbar_x_in, const void* gbar_vec_in, void* gbar_x_out,
                             void* gbar_vec_out, void* vecp_bar, void* o_bar, const void* x, const void* mean,
                             const void* rstd, const void* ln_w, const void* grad_xn, void* gbar_grad_xn,
                             void* x_bar, void* w_bar_rows, void* stream);
/* The same with the incoming vec cotangent as the sum of two buffers (gbar_vec_in + gbar_vec_in2, either
 * NULL = 0): the force-loss adjoint passes the message VJP's d_gvec beside the running vec cotangent, so no
 * separate add launch forms their sum. */
int tmdnet_et_adjoint_epi_ln2(int dtype, int n_nodes, int hidden, const void* gb_o, const void* gb_vecp,
                              const void* grad_x, const void* grad_vec, const void* vecp, const void* o,
                              const void* gbar_x_in, const void* gbar_vec_in, const void* gbar_vec_in2,
                              void* gbar_x_out, void* gbar_vec_out, void* vecp_bar, void* o_bar, const void* x,
                              const void* mean, const void* rstd, const void* ln_w, const void* grad_xn,
                              void* gbar_grad_xn, void* x_bar, void* w_bar_rows, void* stream);

/* ------------------------------------------------------------------------------------------
 * EquivariantScalar output head (reference models/output_modules.py:80-115 with two
 * GatedEquivariantBlocks, models/utils.py:456-522: H -> H/2 with scalar SiLU, then H/2 -> 1;
 * intermediate = hidden; SiLU activations), fused per atom.
 * weights[12] = block 1: vec1_proj.weight [H][H], vec2_proj.weight [H/2][H], update_net[0].weight
 *   [H][2H], update_net[0].bias [H], update_net[2].weight [H][H], update_net[2].bias [H];
 *   block 2: the same six for H/2 (vec2_proj.weight [1][H/2], update_net[2].weight [2][H/2]).
 * x [N][H], vec [N][3][H] -> y [N] (the atom output before std / reduce; the head's "+ 0 * sum vec"
 * term is dropped).  jac_x [N][H], jac_vec [N][3][H] (both NULL or both given): dy_n / d(x_n, vec_n),
 * zero where a vector norm is zero (torch.norm's backward).  H a multiple of 4, <= ~500 (LDS). */
int tmdnet_eq_head_fwd(int dtype, int n_atoms, int hidden, const void* x, const void* vec,
                       const void* const* weights, void* y, void* jac_x, void* jac_vec, void* stream);
/* Backward with weight gradients (training): recomputes the head and writes grad_x, grad_vec
 * (= grad_y[n] * Jacobian) plus the per-atom factors saves[11] of every weight gradient, each a
 * GEMM over atoms (layouts, O = Q = H/2):
 *   0 a1 [N][3][H+O] = [g_vb | g_v2]   -> [dW1; dW2] = a1^T vec           (rows = N*3)
 *   1 gu [N][H], 2 hext [N][2H+1] = [x | vec1 | 1]   -> [dU1 | db1] = gu^T hext
 *   3 go [N][2O], 4 sext [N][H+1] = [s | 1]          -> [dU2 | db2] = go^T sext
 *   5 a2 [N][3][Q+1] = [g_vb2 | 0], 6 v1 [N][3][O]   -> [dV1; dV2] = a2^T v1 (rows = N*3)
 *   7 gu2 [N][Q], 8 h2ext [N][2Q+1]                  -> [dP1 | db1'] = gu2^T h2ext
 *   9 go2 [N][2] = [g_y | 0], 10 s2ext [N][Q+1]      -> [dP2 | db2'] = go2^T s2ext */
int tmdnet_eq_head_bwd_weights(int dtype, int n_atoms, int hidden, const void* x, const void* vec,
                               const void* const* weights, const void* grad_y, void* grad_x,
                               void* grad_vec, void* const* saves, void* stream);
/* Second order of the head's backward (force-matching training; replaces the double differentiation
 * of the gated blocks, reference models/utils.py:492-522 under module.py:130-179's force loss).  For
 * cotangents (tan_x [N][H], tan_vec [N][3][H]; NULL = 0) of (grad_x, grad_vec) = grad_y[n] * J(x, vec):
 *   d_x, d_vec = grad_y[n] * d/dt J(x + t tan_x, vec + t tan_vec)   (Hessian-vector product)
 *   d_grad_y[n] = <tan_x, J_x> + <tan_vec, J_vec>                    (NULL = not written)
 * saves[12] (NULL = no weight terms): the layouts of tmdnet_eq_head_bwd_weights for 2N atoms
 * ([tangent half ; plain half]) plus saves[11] = vv [2][N][3][H] = [vec ; tan_vec]; each weight's
 * second-order term is then one GEMM over 2N (6N) rows, e.g. [dW1; dW2] = a1^T vv. */
int tmdnet_eq_head_hvp(int dtype, int n_atoms, int hidden, const void* x, const void* vec,
                       const void* const* weights, const void* grad_y, const void* tan_x,
                       const void* tan_vec, void* d_x, void* d_vec, void* d_grad_y,
                       void* const* saves, void* stream);
/* The same forward + Jacobian (seeded with grad_y, NULL = 1) on the bf16 MFMA at fp32 accuracy over 16-atom
 * tiles (eq_head_x3.hip): fp32, hidden = 128 only (else TMDNET_UNSUPPORTED).  pieces[10]: the exact
 * three-piece bf16 splits (tmdnet_proj_split_f32 layout [3][N][K]) of [W1; W2] (192 x 128), U1 (128 x 256),
 * U2 (128 x 128), V1 (64 x 64), P1 (64 x 128) and of their transposes P1^T, V1^T, U2^T, U1^T, [W1; W2]^T;
 * vectors[5] = u1b, u2b, p1b, p2w (2 x 64), p2b (block 1 = vec1_proj W1, vec2_proj W2, update_net U1 / U2;
 * block 2 = V1, P1 / P2).  jac_x / jac_vec both or neither; 16-byte aligned rows. */
int tmdnet_eq_head_x3_f32(int n_atoms, int hidden, const void* x, const void* vec, const void* const* pieces,
                          const void* const* vectors, void* y, void* jac_x, void* jac_vec, const void* grad_y,
                          void* stream);
/* The ten piece matrices of tmdnet_eq_head_x3_f32 from the head's 12 weights (tmdnet_eq_head_fwd's order),
 * in ONE launch, packed back to back in that order into pieces_buf (tmdnet_eq_head_x3_pieces_bytes). */
size_t tmdnet_eq_head_x3_pieces_bytes(int hidden);
int tmdnet_eq_head_x3_split_f32(int hidden, const void* const* weights, void* pieces_buf, void* stream);
/* grad_x = grad_y[n] * jac_x[n], grad_vec = grad_y[n] * jac_vec[n] (the head's backward). */
int tmdnet_eq_head_bwd(int dtype, int n_atoms, int hidden, const void* grad_y, const void* jac_x,
                       const void* jac_vec, void* grad_x, void* grad_vec, void* stream);

/* Neighbour embedding aggregation (reference NeighborEmbedding.forward/message,
 *   models/utils.py:73-108):  out[t] = sum_{e in row t, src!=dst} X[src[e]] * W[e] * C[e]
 *   X: [N][H] (ld_x), W: [E][H] (ld_w) = distance_proj(rbf) pre-cutoff, C: [E], out [N][H]. */
int tmdnet_nbr_embed_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                         const int32_t* src, int max_pairs, const void* x, int ld_x, const void* w,
                         int ld_w, const void* cutoff, void* out, int ld_out, const void* x_self,
                         void* out_self, void* stream);
/* Backward: gx[s] (source pass, symmetric list; gx NULL: not computed -- the force pass never needs it),
 * gw[e], gcut[e] (destination pass, every slot < max_pairs written: padding slots zero); overwritten.
 * ld_out / ld_grad_out: row strides of out / grad_out (0 = hidden), so the output can be the right
 * half of the combine Linear's [x | x_nb] input (reference utils.py:108) and its gradient read from
 * that layout in place; x_self / out_self (both or neither): the forward also copies x_self [n][hidden]
 * rows into out_self (stride ld_out), the left half -- the concatenation costs no launch. */
int tmdnet_nbr_embed_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                         const int32_t* src, int max_pairs, const void* x, int ld_x, const void* w,
                         int ld_w, const void* cutoff, const void* grad_out, int ld_grad_out, void* gx,
                         void* gw, void* gcut, void* stream);
/* Second order of the neighbour embedding (force-matching training; replaces autograd's double
 * differentiation of reference utils.py:100-107): the VJP of (gx, gw, gcut) = tmdnet_nbr_embed_bwd(...)
 * for cotangents gg_x [N][H], gg_w [E][H], gg_cut [E] (NULL = 0), with respect to grad_out (d_grad_out
 * [N][H]), x (d_x [N][H], source pass over the reversed edges transpose[e]), w (d_w [E][H]) and the
 * cutoff (d_cut [E]); outputs NULL = not wanted, edge outputs written for every slot < row_ptr[N]. */
int tmdnet_nbr_embed_bwd2(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                          const int32_t* src, const int32_t* transpose, int max_pairs, const void* x,
                          int ld_x, const void* w, int ld_w, const void* cutoff, const void* grad_out,
                          int ld_grad_out, const void* gg_x, const void* gg_w, const void* gg_cut,
                          void* d_grad_out, void* d_x, void* d_w, void* d_cut, void* stream);

/* ------------------------------------------------------------------------------------------
 * TensorNet edge kernels (reference models/tensornet.py:287-332).
 * Tensors are COMPACT and component-major, [9][N][H]: per channel the coefficients
 * c = [i, a01, a02, a12, s00, s11, s01, s02, s12] of X = i Id + A + S (A antisymmetric, S symmetric
 * traceless; reference decompose_tensor, tensornet.py:47-52), rows 0 / 1-3 / 4-8 being the I / A / S
 * parts.  self0_mult >= 1: multiplicity of atom 0's self loop (static_shapes padding emulation,
 * tensornet.py:215-221; 1 = no padding).  If pad_pairs (device int32, the pair count found by
 * tmdnet_nl_build) is non-NULL the multiplicity is computed on the device instead:
 * 1 + max(0, pad_capacity - *pad_pairs) (no host sync: HIP-graph capturable).  Both require the
 * symmetric CSR list.
 * Embedding (replaces TensorEmbedding._get_tensor_messages + the scatter, tensornet.py:295-315):
 *   I/A/S[n] = sum_{edges e with reference edge_index[0]==n} (P[n] + Q[dst]) * W_k[e] * C[e]
 *              * {Id, skew(u[e]), sym(u[e])},  W = [E][3H] = distance_proj1|2|3(rbf) (pre-cutoff),
 *   P = emb(z) Wa^T + b, Q = emb(z) Wb^T  (emb2 split into its two input halves); out [9][N][H]. */
int tmdnet_tn_embed_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                        const int32_t* src, int max_pairs, double self0_mult,
                        const int32_t* pad_pairs, int pad_capacity, const void* P,
                        const void* Q, const void* W, int ld_w, const void* cutoff, const void* unit,
                        void* out, void* stream);
/* Backward: gP, gQ [N][H], gW [E][3H], gcut [E], gunit [E][3] from grad_out [9][N][H]; overwritten. */
int tmdnet_tn_embed_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                        const int32_t* src, int max_pairs, double self0_mult,
                        const int32_t* pad_pairs, int pad_capacity, const void* P,
                        const void* Q, const void* W, int ld_w, const void* cutoff, const void* unit,
                        const void* grad_out, void* gP, void* gQ, void* gW, void* gcut, void* gunit,
                        void* stream);
/* Second order of the embedding (force-matching training through TensorEmbedding, tensornet.py:287-326 under
 * module.py:130-179): for cotangents (tP, tQ, tW, tcut, tunit) of the first backward's outputs (gP, gQ, gW,
 * gcut, gunit), d_grad_out [9][N][H] = J t (the forward's directional derivative) and (dP, dQ, dW [E][3H],
 * dcut, dunit) = H_<grad_out, E> t (the first backward's directional derivative, grad_out fixed): the
 * first-order kernels evaluated on dual numbers.  tW shares W's row stride ld_w; a NULL tangent is zero, a
 * NULL output is not computed; outputs overwritten. */
int tmdnet_tn_embed_bwd2(int dtype, int n_nodes, int hidden, const int32_t* row_ptr, const int32_t* src,
                         int max_pairs, double self0_mult, const int32_t* pad_pairs, int pad_capacity,
                         const void* P, const void* Q, const void* W, int ld_w, const void* cutoff,
                         const void* unit, const void* grad_out, const void* tP, const void* tQ, const void* tW,
                         const void* tcut, const void* tunit, void* d_grad_out, void* dP, void* dQ, void* dW,
                         void* dcut, void* dunit, void* stream);
/* Message (replaces tensor_message_passing, tensornet.py:329-332):
 *   msg[n] = sum_{edges e with edge_index[0]==n} ea[e,h,0] I[m] + ea[e,h,1] A[m] + ea[e,h,2] S[m],
 * m = edge_index[1][e]; edge_attr [E][3H] interleaved (h, component) as reshape(E, H, 3);
 * comp and msg [9][N][H] (the message of compact tensors is compact). */
int tmdnet_tn_message_fwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                          const int32_t* src, int max_pairs, double self0_mult,
                          const int32_t* pad_pairs, int pad_capacity, const void* edge_attr,
                          int ld_ea, const void* comp, void* msg, void* stream);
/* Backward: g_edge_attr [E][3H] (destination pass), g_comp [9][N][H] (source pass); overwritten. */
int tmdnet_tn_message_bwd(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                          const int32_t* src, int max_pairs, double self0_mult,
                          const int32_t* pad_pairs, int pad_capacity, const void* edge_attr,
                          int ld_ea, const void* comp, const void* grad_msg, void* g_edge_attr,
                          void* g_comp, void* stream);
/* The same with g_comp_add ([9][N][H], or NULL) added to g_comp: the gradient the component tensor's
 * other consumer (TensorNet's decompose(msg Y + Y msg), tensornet.py:398-401) contributes, so the
 * autograd engine does not sum the two in a separate launch. */
int tmdnet_tn_message_bwd_add(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                              const int32_t* src, int max_pairs, double self0_mult,
                              const int32_t* pad_pairs, int pad_capacity, const void* edge_attr,
                              int ld_ea, const void* comp, const void* grad_msg, const void* g_comp_add,
                              void* g_edge_attr, void* g_comp, void* stream);
/* Pair-row forms (large systems): the edge factors are functions of |r| only, so the two directions of a
 * pair share one row.  edge_attr / g_edge_attr are [n_pair_slots][3H] in tmdnet_pair_index's numbering
 * (pair_row [E] -> slot, pair_edge [n_pair_slots] -> the slot's canonical edge, src >= dst); edge e reads
 * row pair_row[e].  The backward's destination pass runs per pair (its canonical edge forms the sum over
 * both directions, one write per pair, no atomics; inert slots zeroed); g_edge_attr or g_comp may be NULL
 * (that pass skipped). */
int tmdnet_tn_message_fwd_pairs(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                const int32_t* src, int max_pairs, double self0_mult,
                                const int32_t* pad_pairs, int pad_capacity, const int32_t* pair_row,
                                const void* edge_attr, int ld_ea, const void* comp, void* msg, void* stream);
int tmdnet_tn_message_bwd_pairs(int dtype, int n_nodes, int hidden, const int32_t* row_ptr,
                                const int32_t* src, int max_pairs, double self0_mult,
                                const int32_t* pad_pairs, int pad_capacity, const int32_t* pair_row,
                                const int32_t* pair_edge, int n_pair_slots, const void* edge_attr, int ld_ea,
                                const void* comp, const void* grad_msg, const void* g_comp_add,
                                void* g_edge_attr, void* g_comp, void* stream);

/* TensorNet per-channel node algebra, one fused pass each (replaces the reference's elementwise
 * PyTorch chains).  X / "full" tensors are [N][H][3][3]; compact ones [9][N][H] as above.
 *   op                 a            b             out
 *   TN_PRE             X            -             decomp(X / (|X|^2+1))          tensornet.py:391-392
 *   TN_POST_O3         Y (compact)  msg (compact) decomp(Z)/(|Z|^2+1), Z=msg Y+Y msg  tensornet.py:398-406
 *   TN_POST_SO3        Y            msg           same, Z = 2 Y msg
 *   TN_RESID           X            D (compact)   X/(|X|^2+1) + D + D D           tensornet.py:391,410
 *   TN_NORMS           X            -             [N][3H] = (|I|^2 | |A|^2 | |S|^2)  tensornet.py:230-231
 *   TN_ENORM           c (compact)  -             [N][H] = |I+A+S|^2              tensornet.py:317
 *   TN_EOUT            c (compact)  f [N][H][3]   f_I I + f_A A + f_S S  (full)   tensornet.py:321-326
 * Backward: ga / gb = VJP w.r.t. a / b from grad_out (same layouts as a / b / out); grad_add
 * (optional, layout of a) is added to ga. */
#define TMDNET_TN_PRE 0
#define TMDNET_TN_POST_O3 1
#define TMDNET_TN_POST_SO3 2
#define TMDNET_TN_RESID 3
#define TMDNET_TN_NORMS 4
#define TMDNET_TN_ENORM 5
#define TMDNET_TN_EOUT 6
int tmdnet_tn_node_fwd(int dtype, int op, int n_nodes, int hidden, const void* a, const void* b,
                       void* out, void* stream);
int tmdnet_tn_node_bwd(int dtype, int op, int n_nodes, int hidden, const void* a, const void* b,
                       const void* grad_out, const void* grad_add, void* ga, void* gb,
                       void* stream);
/* Second order of a node pass (force-matching training; replaces autograd's double differentiation of
 * the pass): the VJP of (ga, gb) = tmdnet_tn_node_bwd(a, b, grad_out) for cotangents t_a / t_b (layouts
 * of a / b; NULL = 0) -- d_grad_out = J (t_a, t_b) (layout of out) and (d_a, d_b) = the Hessian of
 * <grad_out, f(a, b)> applied to (t_a, t_b); every output NULL = not computed, written otherwise.
 * (grad_add's derivative is the identity: the caller passes t_a through.)  b / t_b / d_b only for the
 * two-input passes. */
int tmdnet_tn_node_bwd2(int dtype, int op, int n_nodes, int hidden, const void* a, const void* b,
                        const void* grad_out, const void* t_a, const void* t_b, void* d_grad_out, void* d_a,
                        void* d_b, void* stream);

/* SiLU with an optional per-row scale (TensorNet edge MLP `act(linear(.)) * C`,
 * tensornet.py:385-389; the scalar MLPs of the embedding, output and Scalar head).
 *   out[r][c] = silu(x[r][c]) * (row_scale ? row_scale[r] : 1)     (x row stride ld_x, out dense)
 * Backward: grad_x[r][c] = grad_out[r][c] * row_scale[r] * silu'(x[r][c]) (dense);
 *           grad_scale[r] = sum_c grad_out[r][c] * silu(x[r][c]) (optional). */
int tmdnet_silu_fwd(int dtype, int rows, int cols, const void* x, int ld_x, const void* row_scale,
                    void* out, void* stream);
int tmdnet_silu_bwd(int dtype, int rows, int cols, const void* x, int ld_x, const void* row_scale,
                    const void* grad_out, int ld_g, void* grad_x, void* grad_scale, void* stream);
/* Second order of a Linear + SiLU stack (TensorNet's MLPs, tensornet.py:320-323, 381-385, 233, under
 * force-matching training), per layer of the reverse-mode VJP of the first backward (all [rows][cols]):
 *   tmdnet_mlp2_up:   ahat = ghat silu'(pre);  dpre = ghat a silu''(pre), or for the LAST layer (gy non-NULL:
 *     a = gy * scale[r], scale nullable) dpre = ghat gy scale silu''(pre) + sbar[r] gy silu'(pre),
 *     dgy = ahat scale + sbar[r] silu(pre) (nullable), dscale[r] = sum_c ahat gy (nullable); sbar nullable.
 *   tmdnet_mlp2_down: c = dp + dh silu'(pre) (c may alias dp).
 * pre: row stride ld_pre; a: ld_a; the rest contiguous. */
int tmdnet_mlp2_up(int dtype, int rows, int cols, const void* pre, int ld_pre, const void* ghat, const void* a,
                   int ld_a, const void* gy, const void* scale, const void* sbar, void* ahat, void* dpre, void* dgy,
                   void* dscale, void* stream);
int tmdnet_mlp2_down(int dtype, int rows, int cols, const void* pre, int ld_pre, const void* dh, const void* dp,
                     void* c, void* stream);

/* Per-molecule energy (TorchMD_Net.forward, model.py:263-283 with output_modules.py:27-43):
 *   y[b] = *mean + *std * sum_{n: batch[n] = b} x[n],  b < n_mol <= 8192  (std / mean: device
 *   scalars, NULL = 1 / 0; batch int64).  Backward: grad_x[n] = *std * grad_y[batch[n]]. */
int tmdnet_atom_sum_fwd(int dtype, int n_atoms, int n_mol, const void* x, const int64_t* batch,
                        const void* std_, const void* mean, void* y, void* stream);
int tmdnet_atom_sum_bwd(int dtype, int n_atoms, int n_mol, const void* grad_y, const int64_t* batch,
                        const void* std_, void* grad_x, void* stream);

/* Scalar head tail fused with the reduction (output_modules.py:83-105, model.py:263-283):
 *   y[b] = *mean + *std * sum_{n: batch[n] = b} (h[n] . w + *b0),  h [n_atoms][K] (ld_h), n_mol <= 8192
 *   (std / mean / b0: device scalars, NULL = 1 / 0 / 0).  Backward: grad_h[n][k] = *std * grad_y[batch[n]] * w[k]. */
int tmdnet_dot_sum_fwd(int dtype, int n_atoms, int K, const void* h, int ld_h, const void* w, const void* b0,
                       int n_mol, const int64_t* batch, const void* std_, const void* mean, void* y, void* stream);
int tmdnet_dot_sum_bwd(int dtype, int n_atoms, int K, const void* grad_y, const int64_t* batch, int n_mol,
                       const void* std_, const void* w, void* grad_h, void* stream);
/* The same for large systems: the row products over the whole grid into atom_buf [n_atoms] (per-atom
 * h[n].w + b0), then the per-molecule sums (atom_buf NULL: tmdnet_dot_sum_fwd). */
int tmdnet_dot_sum_fwd_atoms(int dtype, int n_atoms, int K, const void* h, int ld_h, const void* w, const void* b0,
                             int n_mol, const int64_t* batch, const void* std_, const void* mean, void* atom_buf,
                             void* y, void* stream);

/* LayerNorm over the last dimension, fp32, C <= 1024 (reference nn.LayerNorm; TensorNet's init_norm /
 * out_norm, models/tensornet.py:232, 322): y = (x - mean) * rstd * w + b, mean / rstd [rows] saved.
 * Backward: grad_x = rstd * (g w - mean(g w) - xhat * mean(g w xhat)) (accumulate: +=, grad_x contiguous);
 * weight / bias gradients as deterministic column sums over the rows (workspace from
 * tmdnet_layernorm_wgrad_workspace_bytes; grad_w or grad_b may be NULL). */
int tmdnet_layernorm_fwd_f32(int rows, int C, const void* x, int ldx, const void* w, const void* b, double eps,
                             void* y, int ldy, void* mean, void* rstd, void* stream);
int tmdnet_layernorm_bwd_f32(int rows, int C, const void* x, int ldx, const void* w, const void* mean,
                             const void* rstd, const void* grad_y, int ldg, void* grad_x, int accumulate,
                             void* stream);
/* Second order (force-matching training through TensorNet's LayerNorms): for cotangents t_gx [rows][C],
 * t_gw [C], t_gb [C] (each nullable) of the first backward's (grad_x, grad_w, grad_b): d_grad_y, d_x [rows][C]
 * (nullable) and t_row [rows][C] (nullable) = rstd (t_gx - mean t_gx - xhat mean(t_gx xhat)), from which the
 * caller forms d_w = colsum(grad_y t_row) (d_b = 0). */
int tmdnet_layernorm_bwd2_f32(int rows, int C, const void* x, int ldx, const void* w, const void* mean,
                              const void* rstd, const void* grad_y, int ldg, const void* t_gx, const void* t_gw,
                              const void* t_gb, void* d_grad_y, void* d_x, void* t_row, void* stream);
size_t tmdnet_layernorm_wgrad_workspace_bytes(int rows, int C);
int tmdnet_layernorm_wgrad_f32(int rows, int C, const void* x, int ldx, const void* mean, const void* rstd,
                               const void* grad_y, int ldg, void* grad_w, void* grad_b, void* workspace,
                               size_t workspace_bytes, void* stream);

/* Pair numbering of a symmetric CSR edge list (for pk_rows above).  Canonical edges are those
 * with src >= dst (self loops and one direction of every pair), numbered row by row in CSR order;
 * pair_row[e] = the pair number of e (the canonical edge's for the other direction), pair_edge[p]
 * = the canonical edge of pair p.  Slots p >= the number of pairs (up to n_pair_slots) and edge
 * slots past *num_pairs (static capacity; num_pairs NULL: row_ptr[n]) get 0.  Requires the
 * transpose map.  sorted_rows != 0 (rows in ascending source order, the brute / shared lists;
 * needs dst) selects a 3-launch closed-form path, else 4 wave-per-row passes.
 * Workspace: tmdnet_pair_index_workspace_bytes(n_nodes). */
size_t tmdnet_pair_index_workspace_bytes(int n_nodes);
int tmdnet_pair_index(int n_nodes, const int32_t* row_ptr, const int32_t* src, const int32_t* dst,
                      const int32_t* transpose, int max_pairs, const int32_t* num_pairs, int sorted_rows,
                      int32_t* pair_row, int32_t* pair_edge, int n_pair_slots, void* workspace,
                      size_t workspace_bytes, void* stream);

/* Grouped small fp32 GEMM on the f32 MFMA (node feature mixes of the ET layer, torchmd_et.py:272-312):
 * up to 4 independent problems in one launch.  Problem i: dims[8i..8i+7] = {M, N, K, lda, ldb, ldc,
 * trans_b, beta}, ptrs[4i..4i+3] = {A, B, bias (nullable), C}:
 *   C[M][N] = beta * C + A[M][K] op(B) + bias[N],  op(B) = B^T for B [N][K] (trans_b) else B [K][N].
 * Requirements: K % 64 == 0, lda % 4 == 0, A 16-byte aligned (and B when trans_b); else
 * TMDNET_UNSUPPORTED (callers use the library GEMM).  Exact fp32 arithmetic. */
int tmdnet_gemm_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream);
/* tmdnet_gemm_f32 with a fused epilogue (a Linear + SiLU stack in one launch per layer, and its
 * backward chain): dims 10 per problem = the 8 of tmdnet_gemm_f32 + (act, ld_x); ptrs 7 per problem =
 * (A, B, bias, C, pre, rscale, dpre).  Per output element: v = A op(B) + bias (+ C if beta);
 * pre != NULL: pre[r][c] = v (row stride ld_x); act = 1: v = silu(v); rscale != NULL: v *= rscale[r];
 * dpre != NULL: v *= silu'(dpre[r][c]) (row stride ld_x); C[r][c] = v.  act in {0, 1}.  Replaces the
 * separate activation launches of the reference's Linear -> act chains (TensorNet edge / embedding
 * MLPs and output head, tensornet.py:233, 320-321, 381-385). */
int tmdnet_gemm_ex_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream);
/* Grouped fp32 weight-gradient GEMM: for each of n_problems (<= 32) C (+)= A^T B + A2^T B2, the sum
 * running over the ROWS of A [K][M] (lda), B [K][N] (ldb) and the optional second segment A2 [K2][M],
 * B2 [K2][N]; C [M][N] (ldc).  ones1 / ones2: column N-1 of B / B2 is a column of ones (not read; with
 * either flag set, a segment without it contributes 0 there), so C's last column is the bias gradient.  dims: 12 ints per problem {M, N, K, K2, lda, ldb, lda2, ldb2,
 * ldc, beta, ones1, ones2}; ptrs: 5 per problem {A, B, A2, B2, C}.  (Every Linear's weight gradient
 * has this shape: the layers' [q|k|v] / vec_proj / o_proj weights in one launch, the head's six.) */
int tmdnet_gemm_tn_f32(int n_problems, const int* dims, const void* const* ptrs, void* stream);
/* The same with a caller-provided workspace: groups with few output tiles over many rows (a 128 x 64
 * weight over 12.5k edge rows is 8 tiles) are split over the rows into S chunks per tile, whose partial
 * tiles a second launch sums in chunk order (deterministic).  workspace_bytes >=
 * tmdnet_gemm_tn_workspace_bytes(n_problems, dims) (0: no split, workspace may be NULL).  ptrs: 6 per
 * problem {A, B, A2, B2, C, Cb}: Cb non-NULL (with ones1 / ones2) receives the ones column, i.e. the
 * bias gradient, as a separate contiguous [M] vector (C then holds the N-1 weight columns). */
size_t tmdnet_gemm_tn_workspace_bytes(int n_problems, const int* dims);
int tmdnet_gemm_tn_f32_ws(int n_problems, const int* dims, const void* const* ptrs, void* workspace,
                          size_t workspace_bytes, void* stream);
/* The same with a device row count per problem: ptrs 7 per problem {A, B, A2, B2, C, Cb, rows}, rows an
 * int32 device scalar (NULL: none): only rows < *rows of each segment are summed.  For the per-edge sums
 * of a static-capacity (HIP-graph) neighbour list, whose padding slots follow the *rows found pairs and
 * contribute zero anyway: the launch's workgroups over padding exit without reading it. */
int tmdnet_gemm_tn_rows_f32_ws(int n_problems, const int* dims, const void* const* ptrs, void* workspace,
                               size_t workspace_bytes, void* stream);
/* Embedding lookups (the forward of nn.Embedding(num_types, H) at z, TorchMD_ET.embedding and
 * NeighborEmbedding.embedding, reference torchmd_et.py:170, utils.py:92; replaces the two index_select
 * gathers): for each of n_tables (<= 4) tables sharing z[n] (int64), outs_t[k][:] = tables_t[z[k]][:]
 * (row strides ld_tables[t] / ld_outs[t], NULL: H; multiples of 4, 16-byte aligned bases) in ONE
 * launch.  An index outside [0, num_types) asserts in the debug build and writes a zero row otherwise. */
int tmdnet_embedding_fwd_f32(int n, int H, int num_types, const int64_t* z, int n_tables,
                             const void* const* tables, const int* ld_tables, void* const* outs,
                             const int* ld_outs, void* stream);
/* Embedding-table gradients (the backward of nn.Embedding(num_types, H) looked up at z, as used by
 * TorchMD_ET.embedding and NeighborEmbedding.embedding, reference torchmd_et.py:170,
 * utils.py:92): for each of n_tables (<= 32) tables sharing the indices z[n] (int64, in [0, num_types)),
 * out_t[m][c] (+= with accumulate) = sum over k with z[k] == m of grads_t[k][c] (row stride ld_grads[t],
 * NULL: H); out_t [num_types][H] contiguous.  fp32, deterministic (one-hot TN GEMM, no atomics). */
int tmdnet_embedding_bwd_f32(int n, int H, int num_types, const int64_t* z, int n_tables,
                             const void* const* grads, const int* ld_grads, void* const* outs, int accumulate,
                             void* stream);
/* The ET dk/dv projection of the pair rows (reference torchmd_et.py:282-291, dk_proj / dv_proj of every
 * layer stacked along N; also its r-derivative and the force-loss adjoint), in two entry points:
 *   tmdnet_proj_split_f32: Wp [3][N][K] (uint16 bf16 bit patterns, 8-byte aligned) = the exact
 *     three-piece bf16 split of W [N][K] (ldw): W = Wp[0] + Wp[1] + Wp[2] elementwise, exactly;
 *   tmdnet_proj_f32: C[M][N] = A[M][K] W[N][K]^T + bias[N] (bias nullable), fp32 in and out, W given
 *     by its split (pieces piece_stride elements apart, so a row slice [r0, r0 + N) of a larger split
 *     is Wp + r0 * K with the larger split's stride).
 * Runs on the bf16 MFMA: A is split the same way in registers and the six products of pieces whose
 * orders sum to <= 2 are accumulated in fp32 -- fp32 GEMM accuracy (not a bf16 result).  Requirements:
 * K = 32 or 64 (split: K % 4 == 0), N % 16 == 0, lda / ldc multiples of 4, 16-byte aligned A / Wp / C /
 * bias; else TMDNET_UNSUPPORTED (callers use the library GEMM).  Replaces the nn.Linear of
 * torchmd_et.py:287-288 over the edges. */
/* Large-row fp32 GEMMs at fp32 accuracy on the bf16 MFMA (the node feature mixes of C5-size systems:
 * EquivariantMultiHeadAttention q/k/v, vec_proj, o_proj Linears and their input gradients,
 * reference torchmd_et.py:273-278, 309; the NeighborEmbedding distance_proj, models/utils.py:98-103):
 *   tmdnet_split_t_f32: Bp [3][N][K] = the exact bf16 pieces of B^T for a [K][N] right operand (ldb);
 *     (a [N][K] Linear weight is split by tmdnet_proj_split_f32);
 *   tmdnet_gemm_x3_f32: C [M][N] = beta C + A [M][K] Bp^T + bias (nullable) -- K % 32 == 0, N % 16 == 0,
 *     16-byte aligned rows / pointers, otherwise TMDNET_UNSUPPORTED (nothing launched). */
int tmdnet_split_t_f32(int N, int K, const void* B, int ldb, void* Bp, void* stream);
int tmdnet_gemm_x3_f32(int M, int N, int K, const void* A, int lda, const void* Bp, const void* bias, void* C,
                       int ldc, int beta, void* stream);
/* tmdnet_gemm_x3_f32 with tmdnet_gemm_ex_f32's epilogue, for the Linear + SiLU stacks of large systems
 * (TensorNet's edge MLP, reference tensornet.py:381-385, over ~1M pair rows at C5; the embedding's scalar
 * MLP tensornet.py:320-321): v = acc + bias (+ C if beta) -> pre[r][c] = v (nullable) -> v = silu(v) if act
 * -> v *= rscale[r] (nullable) -> v *= silu'(dpre[r][c]) (nullable) -> C.  pre / dpre: row stride ldx
 * (>= N, % 4), 16-byte aligned. */
int tmdnet_gemm_x3_ex_f32(int M, int N, int K, const void* A, int lda, const void* Bp, const void* bias, void* C,
                          int ldc, int beta, int act, void* pre, const void* rscale, const void* dpre, int ldx,
                          void* stream);
/* tmdnet_gemm_x3_ex_f32 with the right operand as fp32, split into its exact bf16 pieces inside the kernel
 * while it is staged in LDS (no split launch, no cached pieces): trans_w = 1 -> W [N][K] (a Linear weight,
 * C = A W^T), trans_w = 0 -> W [K][N] (C = A W); ldw % 4 == 0, W 16-byte aligned. */
int tmdnet_gemm_x3w_f32(int M, int N, int K, const void* A, int lda, const void* W, int ldw, int trans_w,
                        const void* bias, void* C, int ldc, int beta, int act, void* pre, const void* rscale,
                        const void* dpre, int ldx, void* stream);
int tmdnet_proj_split_f32(int N, int K, const void* W, int ldw, void* Wp, void* stream);
int tmdnet_proj_f32(int M, int N, int K, const void* A, int lda, const void* Wp, long long piece_stride,
                    const void* bias, void* C, int ldc, void* stream);

/* The ET message with the dk/dv projection FUSED in (reference torchmd_et.py:282-291 + :314-347, the
 * RBF of models/utils.py:272-344): tmdnet_et_message_fwd's outputs without the projection rows.  Per
 * 16-edge tile the fragments of the RBF values of the edges are multiplied on the fp16 MFMA by the
 * layer's weight, held in LDS for the whole launch as the image made by tmdnet_fep_split_f32 (two fp16
 * pieces per value after exact power-of-two scaling: fp32-GEMM accuracy).
 *   tmdnet_fep_split_f32: W [D][R] (ldw) = the layer's [dk | dv] rows in the planar order (dk, then the
 *     x, v1, v2 H-blocks of dv), bias [D] (nullable) -> img (tmdnet_fep_image_bytes(D, R), 16-byte
 *     aligned), wsc [D] (accumulator scale per row), bias_out [D].
 *   tmdnet_fep_frags_f32: the RBF (and d RBF / d r) MFMA fragments of `rows` projection rows (pair rows)
 *     at distances r_rows [rows]: frags [rows][4][R] fp16 (tmdnet_fep_frags_bytes; f and f' in two pieces
 *     each), dscale [rows] (the derivative's power-of-two scale).  mu / beta: the RBF means / betas
 *     (gauss: offsets / coeff[0]).  Once per evaluation: every layer reads the same fragments.
 *   tmdnet_et_fused_fwd_f32: fp32 only; H = 128, heads = 8 (d = 16), R = 32 or 64, both projections
 *     present (distance_influence "both"), SiLU activations; edge e reads fragment row frag_rows[e] (its
 *     pair row; n_frag_rows rows); v in the planar layout when flags carries TMDNET_ET_V_PLANAR, else the
 *     reference's per-head [x|v1|v2] interleave; q / k / v / vec_in / x_out / vec_out / frags 16-byte
 *     aligned with leading dimensions % 4 == 0; vec_in nullable (layer 0).  Else TMDNET_UNSUPPORTED.  One
 *     workgroup per CU (its LDS), deterministic, no atomics on outputs. */
size_t tmdnet_fep_image_bytes(int D, int R);
int tmdnet_fep_split_f32(int D, int R, const void* W, int ldw, const void* bias, void* img, void* wsc,
                         void* bias_out, void* stream);
size_t tmdnet_fep_frags_bytes(long long rows, int R);
int tmdnet_fep_frags_f32(long long rows, int R, const void* r_rows, const void* mu, const void* beta,
                         double cutoff_lower, double cutoff_upper, int rbf_type, void* frags, void* dscale,
                         void* stream);
int tmdnet_et_fused_fwd_f32(int n_nodes, int hidden, int heads, int num_rbf, const int32_t* row_ptr,
                            const int32_t* src, int max_pairs, const void* q, int ld_q, const void* k, int ld_k,
                            const void* v, int ld_v, const void* vec_in, const void* cutoff, const void* unit,
                            const int32_t* frag_rows, const void* frags, long long n_frag_rows, const void* img,
                            const void* wsc, const void* bias, void* x_out, void* vec_out, int flags, void* stream);

/* The fused message's first-order backward for the force pass ("dr mode", reference: the autograd of
 * torchmd_et.py:282-291, :314-347 through f = rbf(r)): d pre / d r = W f'(r) is formed on the MFMA per
 * tile beside the projection (both from the tmdnet_fep_split_f32 image and the tmdnet_fep_frags_f32
 * fragments), and the projection gradient is contracted with it in registers: gdist[e] = <g_pre,
 * d pre / d r>.  Outputs as tmdnet_et_message_bwd in dr mode (destination pass: gq, gcut, gunit, gdist;
 * source pass over the reversed edges: gk, gv (v's layout), gvec_in), with its accumulate bits
 * (TMDNET_ACC_VEC_RESIDUAL / _EDGE / _GRADS, and TMDNET_ET_V_PLANAR for the layout); rows
 * [row_ptr[n], max_pairs) of gcut / gunit / gdist are set to 0.  workspace: tmdnet_et_fused_bwd_workspace_bytes
 * (max_pairs) bytes (the per-head-slice edge sums; 0 = none needed).  Same envelope as
 * tmdnet_et_fused_fwd_f32; the gradient buffers 16-byte aligned; requires a pair-symmetric edge list
 * (tmdnet_et_message_bwd's precondition). */
size_t tmdnet_et_fused_bwd_workspace_bytes(int max_pairs);
int tmdnet_et_fused_bwd_f32(int n_nodes, int hidden, int heads, int num_rbf, const int32_t* row_ptr,
                            const int32_t* src, int max_pairs, const void* q, int ld_q, const void* k, int ld_k,
                            const void* v, int ld_v, const void* vec_in, const void* cutoff, const void* unit,
                            const int32_t* frag_rows, const void* frags, const void* dscale, long long n_frag_rows,
                            const void* img, const void* wsc, const void* bias, const void* grad_x,
                            const void* grad_vec, void* gq, void* gk, void* gv, void* gvec_in, void* gcut,
                            void* gunit, void* gdist, int accumulate, void* workspace, size_t workspace_bytes,
                            void* stream);

/* The neighbour embedding with distance_proj FUSED in (reference NeighborEmbedding, models/utils.py:90-108):
 * tmdnet_nbr_embed_fwd's output with W = distance_proj(rbf) formed per 16-edge tile on the fp16 MFMA from
 * the tmdnet_fep_frags_f32 fragments and the tmdnet_fep_split_f32 image of distance_proj (D = hidden
 * rows, its bias) -- no E x hidden rows:
 *   out[t] = sum_{e in row t, src[e] != t} x[src[e]] * (W f(r_e) + b) * cutoff[e]   (row stride ld_out),
 * and with x_self / out_self (both or neither) the [x_self | x_nb] concatenation as tmdnet_nbr_embed_fwd.
 * The force pass's backward ("dr mode", first order, no parameter or x gradients) -- per edge
 *   gcut[e] = sum_h grad_out[t][h] x[s][h] (W f + b)[h],  gdist[e] = cutoff[e] sum_h grad_out[t][h] x[s][h] (W f')[h]
 * (0 for self edges), written (or added with TMDNET_ACC_EDGE; written: rows [row_ptr[n], max_pairs) set to 0).
 * fp32; hidden = 128, num_rbf 32 or 64; x / img / frags / out / grad_out 16-byte aligned, strides % 4 == 0;
 * else TMDNET_UNSUPPORTED. */
int tmdnet_nbr_fused_fwd_f32(int n_nodes, int hidden, int num_rbf, const int32_t* row_ptr, const int32_t* src,
                             int max_pairs, const void* x, int ld_x, const void* cutoff, const int32_t* frag_rows,
                             const void* frags, long long n_frag_rows, const void* img, const void* wsc,
                             const void* bias, void* out, int ld_out, const void* x_self, void* out_self,
                             void* stream);
int tmdnet_nbr_fused_bwd_f32(int n_nodes, int hidden, int num_rbf, const int32_t* row_ptr, const int32_t* src,
                             int max_pairs, const void* x, int ld_x, const void* cutoff, const int32_t* frag_rows,
                             const void* frags, const void* dscale, long long n_frag_rows, const void* img,
                             const void* wsc, const void* bias, const void* grad_out, int ld_grad_out, void* gcut,
                             void* gdist, int accumulate, void* stream);

/* Energy + force MSE training loss (reference LNNP.step, module.py:130-179, mean reductions):
 *   out[0] = w1 * mean((a1 - b1)^2) + w2 * mean((a2 - b2)^2)   over n1 / n2 elements (one launch),
 * and its backward d1 = g w1 2 (a1 - b1) / n1, d2 = g w2 2 (a2 - b2) / n2 with g = grad_out[0] read
 * on the device (d1 / d2 nullable). */
int tmdnet_mse2_fwd(int dtype, int n1, const void* a1, const void* b1, double w1, int n2, const void* a2,
                    const void* b2, double w2, void* out, void* stream);
int tmdnet_mse2_bwd(int dtype, int n1, const void* a1, const void* b1, double w1, int n2, const void* a2,
                    const void* b2, double w2, const void* grad_out, void* d1, void* d2, void* stream);

/* Library identification (for load checks). */
const char* tmdnet_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* TMDNET_H */
