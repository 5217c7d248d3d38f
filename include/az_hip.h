/* libaz_hip.so — C-ABI of the MI355X (gfx950) board-evaluation hot path of
 * andrpac/alphazero-gnn: the Connect4/TicTacToe conv trunk + policy/value heads,
 * the GNN message-passing layers of gnn_utils.py, their backward pass and Adam.
 *
 * Conventions
 *   - Every pointer except the ones documented as host pointers is a DEVICE pointer
 *     (HBM), caller-allocated.  No entry point allocates, frees or synchronises, so a
 *     caller may capture them into a hipGraph.
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream).
 *   - All arithmetic is fp32 (the reference runs torch fp32: SURVEY.md §0.8); GEMM-shaped
 *     work runs on v_mfma_f32_32x32x2_f32, everything else on the VALU.
 *   - Return value: AZ_OK (0) or a negative AZ_E* code; az_last_error() explains it.
 *   - Layouts are the reference's: nn.Linear weights [out][in] row-major, conv weights
 *     [Cout][Cin][3][3], features the NCHW flatten c*n*n + x*n + y
 *     (connect4/Connect4Net.py:42-49).
 *
 * Each entry point names the reference interface it replaces (path:line in the
 * reference tree).  The Python binding (ctypes) is alphazero-gnn_amd/azhip/_lib.py;
 * INTEGRATION.md shows the reference-side binding.
 */
#ifndef AZ_HIP_H
#define AZ_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AZ_ABI_VERSION 2

#define AZ_OK 0
#define AZ_EINVAL (-1)     /* bad shape / null pointer / misaligned buffer */
#define AZ_ELAUNCH (-2)    /* a kernel launch failed (hipGetLastError) */
#define AZ_EDEVICE (-3)    /* no gfx950 device / HIP runtime error */

#define AZ_ACT_NONE 0
#define AZ_ACT_RELU 1
#define AZ_ACT_SIGMOID 2
#define AZ_ACT_TANH 3
#define AZ_ACT_DRELU 4     /* backward of ReLU: v * (G[i][j] > 0), G = saved activation */

int az_abi_version(void);
const char* az_last_error(void);
/* Checks that the current HIP device is a gfx950 (MI355X); returns AZ_OK or AZ_EDEVICE. */
int az_check_device(void);
/* Zero-copy host staging: fine-grained pinned host memory mapped at the same address on the
 * device (a kernel may read / write it directly; host sees device stores after a stream
 * synchronise).  Returns NULL on failure (az_last_error says why).  No reference counterpart:
 * it replaces the .cpu() / torch.FloatTensor round trips of the batch-1 predict
 * (connect4/Connect4GNN.py:59-84) with in-place reads and writes by the kernels. */
void* az_host_alloc(size_t bytes);
int az_host_free(void* p);

/* ---------------------------------------------------------------------------------
 * Dense fp32 GEMM with fused epilogue:  C = epi(op(A) . op(B))     (MFMA 32x32x2 f32;
 * M <= 8 with a K-major B dispatches to a weight-streaming GEMV kernel).
 * Replaces every nn.Linear of the path (gnn_utils.py:11-28,101-105, Connect4Net.py:21-25,
 * TicTacToeNet.py:21-26) and, with the transposed layouts, their weight/input gradients.
 *   A(i,k) = a_kmajor ? A[r(i)*lda + k] : A[k*lda + i]      r(i) = a_rows ? a_rows[i] : i
 *            (k >= K0 reads A2[r(i)*lda2 + k-K0] when A2 != NULL: concatenation [A | A2]
 *             along K, i.e. torch.cat([t, agg], dim=1) of gnn_utils.py:31,68)
 *   B(k,j) = b_kmajor ? B[j*ldb + k] : B[q(k)*ldb + j]       q(k) = b_rows ? b_rows[k] : k
 *            (b_kmajor = nn.Linear weight [N][K]; b_rows gathers rows of an N-major B)
 *   v      = act(sum_k A(i,k) B(k,j) + bias[j])     (AZ_ACT_DRELU: v * (G[i*ldg+j] > 0))
 *   C2[i*ldc2 + j] = v                                        when C2 != NULL
 *   v      = R ? R[c(i)*ldr + j] + (G ? G[i*ldg + j] : 1) * v : v   (gated residual,
 *            gnn_utils.py:71)
 *   C[c(i)*ldc + j] = v + beta * C[c(i)*ldc + j]             c(i) = c_rows ? c_rows[i] : i
 * ws/ws_bytes: optional device workspace; when the tile grid cannot fill the GPU the K loop is
 * split over workgroups and the fp32 partial slabs (splits*M*N*4 bytes) are reduced in a
 * fixed order (results are deterministic run to run).
 * Requirements: K % 4 == 0 when an operand is K-major; lda, lda2, ldb % 4 == 0 and 16-byte
 * aligned A/A2/B; K0 % 4 == 0; a_rows only with a_kmajor, b_rows only with !b_kmajor;
 * round_up(M, 4) <= lda when !a_kmajor; round_up(N, 4) <= ldb when !b_kmajor.
 * --------------------------------------------------------------------------------- */
typedef struct az_gemm_desc {
  int M, N, K;
  const float* A; int lda; int a_kmajor;
  const float* A2; int lda2; int K0;
  const int* a_rows;
  const float* B; int ldb; int b_kmajor;
  const int* b_rows;
  const float* bias;
  int act;
  const float* R; int ldr;
  const float* G; int ldg;
  float beta;
  float* C; int ldc;
  const int* c_rows;
  float* C2; int ldc2;
  void* ws; size_t ws_bytes;
} az_gemm_desc;

int az_gemm_f32(const az_gemm_desc* d, void* stream);

/* MFMA products per fp32 product that az_gemm_f32 runs for a plain K-major M x N x K GEMM with
 * ws_bytes of workspace: 3 = the fp16 form (each operand row scaled by a power of two and split
 * into two fp16 terms, three products on v_mfma_f32_32x32x16_f16: M > 64, K >= 1024, N >= 256,
 * room for A's row scales), 6 = the bf16 form (three bf16 terms, six products), 1 = an fp32
 * MFMA tile, 0 = the fp32 GEMV (M <= 8).  For rooflines and reports; no GPU work. */
int az_gemm_form(int M, int N, int K, size_t ws_bytes);

/* ---------------------------------------------------------------------------------
 * Connect4Net trunk, connect4/Connect4Net.py:42-49 (== Connect4GNNWrapper.extract_features,
 * connect4/Connect4GNN.py:31-46 in eval mode): conv1 3x3 p1 + ReLU -> conv2 3x3 p1 + ReLU ->
 * NCHW flatten, fused in one kernel (conv1 in LDS, conv2 as an implicit GEMM on MFMA 16x16x4).
 *   boards  int8 [B][7][7] in {-1,0,1} (axis 0 = column x, axis 1 = row y)
 *   feat    fp32 [B][3136]
 * --------------------------------------------------------------------------------- */
int az_c4_trunk_fwd(const int8_t* boards, int B,
                    const float* conv1_w, const float* conv1_b,
                    const float* conv2_w, const float* conv2_b,
                    float* feat, void* stream);

/* 3x3 conv (stride 1, padding `pad` in {0,1}) + ReLU on NCHW input; `in` is int8 boards
 * [B][H][W] (Cin must be 1) when in_int8 != 0, else fp32 [B][Cin][H][W].
 * TicTacToeNet conv1..conv3, tictactoe/TicTacToeNet.py:33-35. */
int az_conv3x3_relu_fwd(const void* in, int in_int8, int B, int Cin, int H, int W,
                        const float* w, const float* b, int Cout, int pad,
                        float* out, void* stream);

/* Policy/value heads: logits = hp . wp^T + bp  -> log_softmax;  v = tanh(hv . wv^T + bv).
 * Connect4GNN.py:48-57 (hp = hv = features, K = 3136) and the last layers of
 * TicTacToeGNN.py:36-45 (hp = relu(fc1), hv = relu(fc2), K = 512).  A <= 32.
 *   logp [B][A], pi [B][A] = exp(logp) (may be NULL), v [B].
 * ws: device scratch of az_heads_ws_bytes(B, K, A) bytes (per-chunk partial dot products,
 * summed in a fixed order). */
size_t az_heads_ws_bytes(int B, int K, int A);
int az_heads_fwd(const float* hp, int ldhp, const float* hv, int ldhv, int B, int K,
                 const float* wp, const float* bp, int A, const float* wv, const float* bv,
                 float* logp, float* pi, float* v, void* ws, size_t ws_bytes, void* stream);

/* Connect4 trunk and policy/value heads in one call: az_c4_trunk_fwd then az_heads_fwd on the
 * feature rows (Connect4Net.py:42-60; Connect4GNN.py:48-57), bit-identical to that pair.  For
 * B <= 320 and A <= 8 it is ONE launch (the heads read the features from the trunk's LDS tile);
 * otherwise the two launches, with ws >= az_heads_ws_bytes(B, 3136, A).  feat [B][3136] is
 * written either way; boards may be az_host_alloc memory (read in place). */
int az_c4_trunk_heads_fwd(const int8_t* boards, int B, const float* conv1_w, const float* conv1_b,
                          const float* conv2_w, const float* conv2_b, const float* wp,
                          const float* bp, int A, const float* wv, const float* bv, float* feat,
                          float* logp, float* pi, float* v, void* ws, size_t ws_bytes,
                          void* stream);

/* The whole Connect4 leaf evaluation of MCTS.search (MCTS.py:169-174 via Connect4GNN.py:59-120:
 * predict and predict_with_gnn of the same boards) as ONE host call with direct launches:
 * trunk + standard heads (az_c4_trunk_heads_fwd), then output_transform + heads on the same
 * features (az_transform_heads_fwd).  Outputs are bit-identical to those calls.  Built for the
 * batch-1 path, where a hipGraph replay costs more host time than these 4 launches. */
typedef struct az_c4_eval {
  const float* conv1_w; const float* conv1_b; const float* conv2_w; const float* conv2_b;
  const float* fc_policy_w; const float* fc_policy_b; const float* fc_value_w;
  const float* fc_value_b;
  int A;                                   /* actions (fc_policy rows) */
  const float* ot0_w; const float* ot0_b;  /* output_transform.0 [3136][3136], [3136] */
  const float* ot2_w; const float* ot2_b;  /* output_transform.2; all four NULL: no GNN tail */
  int max_B;                               /* capacity of the scratch below */
  float* feat; float* hidden; float* y;    /* device [max_B][3136] each (hidden/y: GNN only) */
  float* logp; float* glogp;               /* device [max_B][A] */
  void* ws; size_t ws_bytes;               /* >= az_transform_heads_ws_bytes(max_B, 3136, A) */
  /* Optional (both NULL: four launches).  The batch <= 2 evaluation in ONE launch
   * (c4_leaf_kernel, az_gemm.hip): sync = device int[4096], zeroed once by the caller and left
   * zero by every launch; err = host-visible int (az_host_alloc) the launch sets to 1 if its
   * in-kernel hand-over timed out -- the outputs are then invalid: zero sync and *err, and call
   * again without them.  One evaluation at a time per sync buffer. */
  int* sync; int* err;
} az_c4_eval;
/* v != NULL: standard heads into pi [B][A] (may be NULL) and v [B];  gv != NULL: the GNN tail
 * into gpi / gv.  boards, pi, v, gpi, gv may be az_host_alloc memory.  With v == NULL (the
 * batched predict_with_gnn alone) and registered output_transform weights, the trunk writes
 * output_transform.0's operand already split for the fp16-form GEMM and that GEMM's split-K
 * reduce writes output_transform.2's, both into the last az_transform_heads_ws_bytes-sized
 * region of e->ws; the GNN tail runs as az_transform_heads_fwd with y = NULL (e->y is not
 * written for B > 8), so the outputs are bit-identical to az_c4_trunk_fwd +
 * az_transform_heads_fwd(y = NULL).  Both v and gv above 320 rows (predict_both): the same
 * hand-off, and the trunk kernel that writes the split operand also forms the standard heads from
 * the rows in its LDS tile -- bit-identical to az_heads_fwd on feat.  e->feat and e->hidden are
 * scratch: above 64 rows, when output_transform.0 / .2 take the pre-split operands for certain
 * (registered weights, their planes cached) and nothing else reads the fp32 rows, those rows are
 * not written. */
int az_c4_eval_fwd(const az_c4_eval* e, const int8_t* boards, int B, float* pi, float* v,
                   float* gpi, float* gv, void* stream);

/* Per-row GNN evaluation tail: output_transform then the heads, i.e. gnn_utils.py:115 (in the
 * 1-row form of Connect4GNN.py:108-111, where the layers are the identity, gnn_utils.py:35-36)
 * followed by Connect4GNN.py:48-57 -- the batched predict_with_gnn after extract_features:
 *   hidden = relu(x W0^T + b0);  y = hidden W2^T + b2;  logp = log_softmax(y wp^T + bp);
 *   pi = exp(logp) (may be NULL);  v = tanh(y wv^T + bv).
 * x, hidden, y: [B][F]; W0, W2: [F][F] (nn.Linear layout); wp [A][F]; wv [1][F]; A <= 32.
 * When the second GEMM is split over K, its slab reduction, bias, the store of y and the heads'
 * dot products run in one pass (y is not re-read); results equal az_gemm_f32 + az_heads_fwd
 * bit for bit.  ws: >= az_heads_ws_bytes(B, F, A) rounded up to 256 B; az_transform_heads_ws_bytes
 * leaves room for the split-K slabs (a smaller workspace only limits the K split).
 * y may be NULL when only the heads are wanted (the evaluators): y is then never written -- on
 * the fp16-form split-K tiles (A <= 8, F % 32 == 0) every block folds its tile of y (+ b in its
 * first k split) into per-row dot products with wp / wv, heads_tiles_finalize_kernel sums them in
 * tile order (the heads are linear in y); other shapes form y in workspace scratch
 * (az_transform_heads_ws_bytes includes it).  Those results are the same function to fp32
 * rounding, not bit-identical to the y != NULL path (tests/test_gpu_kernels.py bounds it). */
size_t az_transform_heads_ws_bytes(int B, int F, int A);
/* Its second half alone: y = x W^T + b, then the heads of y (same fusion, same workspace). */
int az_linear_heads_fwd(const float* x, int B, int F, const float* w, const float* b,
                        const float* wp, const float* bp, int A, const float* wv, const float* bv,
                        float* y, float* logp, float* pi, float* v, void* ws, size_t ws_bytes,
                        void* stream);
int az_transform_heads_fwd(const float* x, int B, int F, const float* w0, const float* b0,
                           const float* w2, const float* b2, const float* wp, const float* bp,
                           int A, const float* wv, const float* bv, float* hidden, float* y,
                           float* logp, float* pi, float* v, void* ws, size_t ws_bytes,
                           void* stream);

/* ---------------------------------------------------------------------------------
 * GNN message passing (gnn_utils.py:5-74) over a destination-sorted CSR graph.
 * The reference's star (row 0 = destination, rows 1..N-1 = sources) is the CSR with
 * rowptr = [0, N-1, N-1, ...], col = [1..N-1]; the synthetic grid has one segment per node.
 * --------------------------------------------------------------------------------- */
typedef struct az_graph {
  int V, E;
  const int* rowptr;    /* [V+1] */
  const int* col;       /* [E] source node of edge e (sorted by destination) */
  const int* edge_dst;  /* [E] destination node of edge e */
  int D;                /* number of destinations with >= 1 in-edge */
  const int* dst_rows;  /* [D] those destinations (ascending) */
  /* backward only (may be NULL for forward use): */
  const int* src_rowptr;  /* [V+1] reverse CSR by source */
  const int* src_edges;   /* [E] edge ids grouped by source (ascending within a source) */
  const int* dst_index;   /* [V] compact destination index, -1 when no in-edge */
  int max_deg;            /* max in-degree (backward supports <= 256); only picks kernels: an
                             understated value is slower, never wrong (edges are not dropped) */
  int band;               /* max |src - dst| over the edges when the caller knows it, else 0.
                             Eval-mode layers on F = 64, H = 128 graphs with 0 < band <= 32 (the
                             row-major grid: 32) run the band kernel (az_gnn_layer_infer); a
                             source outside the claimed band takes a slow path, never wrong */
} az_graph;

typedef struct az_gnn_layer_w {     /* GNNLayer parameters, state_dict order */
  const float* att_w1; const float* att_b1;   /* attention.0  [H][2F], [H] */
  const float* att_w2; const float* att_b2;   /* attention.2  [1][H],  [1] */
  const float* upd_w1; const float* upd_b1;   /* update_net.0 [F][2F], [F] */
  const float* upd_w2; const float* upd_b2;   /* update_net.2 [F][F],  [F] */
  const float* gate_w; const float* gate_b;   /* gate.0       [F][2F], [F] */
} az_gnn_layer_w;

typedef struct az_gnn_layer_grads { /* gradients, same layout as az_gnn_layer_w (written) */
  float* att_w1; float* att_b1; float* att_w2; float* att_b2;
  float* upd_w1; float* upd_b1; float* upd_w2; float* upd_b2;
  float* gate_w; float* gate_b;
} az_gnn_layer_grads;

/* alpha[e] = sigmoid(w2 . relu(P[dst(e)][2q] + P[col(e)][2q+1] + b1) + b2)
 * the factored attention MLP of GNNLayer.compute_attention (gnn_utils.py:30-32,48-55):
 * W1 [t; x] = W1[:, :F] t + W1[:, F:] x, so both halves are projected once per NODE.
 * P [V][2H] (row stride ldp) interleaves them: P[v][2q] = W1[q, :F].x_v,
 * P[v][2q+1] = W1[q, F:].x_v, which is exactly the GEMM x . W1'^T with W1 [H][2F] read as
 * [2H][F] (row stride F).  H % 2 == 0. */
int az_gnn_attn_score_fwd(const az_graph* g, const float* P, int ldp, int H,
                          const float* b1, const float* w2, const float* b2,
                          float* alpha, void* stream);

/* agg[d] = sum_{e in seg(d)} a'_e x[col(e)],  a' = a / sum(a) when sum(a) > 0
 * (gnn_utils.py:57-65), for the D destinations g->dst_rows (D == V means every row);
 * other rows of agg are not written.  Edges are summed in CSR order (deterministic).
 * x, agg: [V][F] with row strides ldx, ldagg; F % 4 == 0. */
int az_gnn_aggregate_fwd(const az_graph* g, const float* x, int ldx, int F,
                         const float* alpha, float* agg, int ldagg, void* stream);

/* One full GNNLayer.forward (gnn_utils.py:34-74) generalised per destination:
 * x_out[d] = x[d] + sigmoid(Wg[x_d;agg_d]+bg) * (Wu2 relu(Wu1[x_d;agg_d]+bu1)+bu2) for the D
 * destinations, x_out[v] = x[v] for every other row (a 1-row GNNLayer input is returned
 * unchanged, gnn_utils.py:35-36).  x_out may not alias x.  `ws` is a device workspace of
 * az_gnn_layer_ws_bytes() bytes; when `save` is non-NULL the activations the backward
 * pass needs are kept in it (see az_gnn_layer_bwd). */
size_t az_gnn_layer_ws_bytes(int V, int E, int D, int F, int H);
int az_gnn_layer_fwd(const az_graph* g, const float* x, int F, int H, const az_gnn_layer_w* w,
                     float* x_out, void* ws, size_t ws_bytes, void* stream);

/* Inference form of az_gnn_layer_fwd (eval mode: same function, nothing kept for a backward
 * pass).  F == 64, H == 128:
 *  - 0 < g->band <= 32 (node-ordered band graphs: the synthetic grid, config 5): ONE band
 *    kernel launch (after a 221 KB weight split into ws): per 64-destination tile, projections,
 *    attention scores, normalised aggregation, gate / update MLPs and the gated residual in LDS /
 *    registers on fp32-accurate bf16x3 MFMAs; x and the source projection of each node are read /
 *    computed once, in a rolling window (gnn_utils.py:30-74);
 *  - else 0 < g->max_deg <= 4: ONE source-projection GEMM (Ps = x W1[:, F:]^T, [V][H] in ws) plus
 *    ONE fused kernel per 64-destination tile;
 *  - other shapes run az_gnn_layer_fwd.
 * ws >= az_gnn_layer_infer_ws_bytes(g, F, H). */
size_t az_gnn_layer_infer_ws_bytes(const az_graph* g, int F, int H);
int az_gnn_layer_infer(const az_graph* g, const float* x, int F, int H, const az_gnn_layer_w* w,
                       float* x_out, void* ws, size_t ws_bytes, void* stream);
/* The network's LAST layer followed by output_transform (gnn_utils.py:87-117 in eval mode:
 * y = output_transform(GNNLayer(x)), output_transform = Linear + ReLU + Linear on every row).
 * On band graphs (see az_gnn_layer_infer) ONE launch: the tile's layer output never leaves LDS
 * and only y is written.  Otherwise az_gnn_layer_infer into ws, then az_mlp2_fwd.
 * ot_w0 / ot_w2: [F][F] nn.Linear weights; y may not alias x.
 * ws >= az_gnn_layer_ot_infer_ws_bytes(g, F, H). */
size_t az_gnn_layer_ot_infer_ws_bytes(const az_graph* g, int F, int H);
int az_gnn_layer_ot_infer(const az_graph* g, const float* x, int F, int H,
                          const az_gnn_layer_w* w, const float* ot_w0, const float* ot_b0,
                          const float* ot_w2, const float* ot_b2, float* y, void* ws,
                          size_t ws_bytes, void* stream);
/* The two launches of the fused path, separately (profiling / callers that keep Ps):
 * Ps [V][H] = x W1[:, F:]^T, then the fused layer kernel given Ps (copies non-destination rows
 * of x to x_out first when D < V).  Fused shapes only (AZ_EINVAL otherwise). */
int az_gnn_source_proj_fwd(const az_graph* g, const float* x, int F, int H,
                           const az_gnn_layer_w* w, float* Ps, void* ws, size_t ws_bytes,
                           void* stream);
int az_gnn_layer_fused_fwd(const az_graph* g, const float* x, const float* Ps, int F, int H,
                           const az_gnn_layer_w* w, float* x_out, void* stream);

/* GNNLayer's gated node update on its own (gnn_utils.py:18-28 gate / update_net, :67-74), for a
 * caller that computes the attention and the aggregation itself (SURVEY §8b
 * az_gnn_node_update_fwd).  The destinations are dst_rows[0..D) -- the rows the reference's
 * destination mask selects; D == V with dst_rows NULL means every row:
 *   c = [x_d ; agg_d],  gate = sigmoid(Wg c + bg),  u1 = relu(Wu1 c + bu1),  u = Wu2 u1 + bu2,
 *   x_out[d] = x[d] + gate * u,  x_out[v] = x[v] on every other row.
 * x, agg, x_out: [V][F] (agg read on the destination rows only); x_out may not alias x;
 * F % 16 == 0.  gate_w / upd_w1: [F][2F], upd_w2: [F][F] (nn.Linear layout).
 * save: [3][D][F] written (gate, u1, u), read by az_gnn_node_update_bwd.
 * ws >= az_gnn_node_update_ws_bytes(D, F).  The same GEMMs, in the same order, as the update
 * inside az_gnn_layer_fwd. */
size_t az_gnn_node_update_ws_bytes(int D, int F);
int az_gnn_node_update_fwd(const float* x, const float* agg, int V, int F, int D,
                           const int* dst_rows, const float* gate_w, const float* gate_b,
                           const float* upd_w1, const float* upd_b1, const float* upd_w2,
                           const float* upd_b2, float* x_out, float* save, void* ws,
                           size_t ws_bytes, void* stream);

/* output_transform, gnn_utils.py:101-105,115: y = W2 relu(W0 x + b0) + b2 on M rows.
 * hidden: [M][F] scratch (kept for the backward pass); ws: optional split-K workspace. */
int az_mlp2_fwd(const float* x, int M, int F, const float* w0, const float* b0,
                const float* w2, const float* b2, float* hidden, float* y,
                void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Backward pass (Connect4GNN.py:150-156,187-197 / TicTacToeGNN.py:217-264), deterministic:
 * every reduction runs in a fixed order, no float atomics.
 * --------------------------------------------------------------------------------- */
/* d loss / d logits and d loss / d tanh-input of the value head for
 * l = -sum(pi*logp)/B_norm + sum((z-v)^2)/B_norm (Connect4GNN.py:150-152).
 * loss_rows (nullable): [B][2] per-row (policy, value) loss terms. */
int az_heads_loss_bwd(const float* logp, const float* v, const float* target_pi,
                      const float* target_v, int B, int A, int B_norm, float* dlogits,
                      float* dvpre, float* loss_rows, void* stream);
/* Heads backward: dwp/dbp/dwv/dbv (nullable as a group) and dhp/dhv (nullable as a pair;
 * dhv == dhp sums both heads into one buffer, the Connect4 case hp == hv).
 * ws >= az_colsum_ws_bytes(B, A+1) bytes when weight grads are requested. */
int az_heads_bwd(const float* dlogits, const float* dvpre, const float* hp, int ldhp,
                 const float* hv, int ldhv, int B, int K, const float* wp, int A,
                 const float* wv, float* dwp, float* dbp, float* dwv, float* dbv,
                 float* dhp, int lddhp, float* dhv, int lddhv, void* ws, size_t ws_bytes,
                 void* stream);
/* out[j] = beta*out[j] + sum_i X[i][j] (bias gradients), fixed-order two-pass reduce. */
size_t az_colsum_ws_bytes(int R, int C);
int az_colsum(const float* X, int R, int C, int ldx, float* out, float beta, void* ws,
              size_t ws_bytes, void* stream);
/* Dropout (Connect4Net.py:52, F.dropout semantics y = x * keep / (1-p)): a counter-based
 * keep mask (mask[i] = 1 with probability 1-p, reproducible from `seed`), and y = mask ? x*scale : 0
 * (forward with scale = 1/(1-p); backward on the gradient with the same mask). */
int az_dropout_mask(uint8_t* mask, int64_t n, double p, uint64_t seed, void* stream);
int az_mask_scale(const float* x, const uint8_t* mask, float scale, int64_t n, float* y,
                  void* stream);
/* Conv trunk backward helpers (3x3, stride 1; pad in {0,1}):
 *   dz[b*HW+p][c] = dy[b][c*HW+p] * (mask ? mask*scale : 1) * (y > 0)   NCHW -> position-major
 *   cols[(b,y,x)][c*9+kh*3+kw] = in[b][c][y+kh-pad][x+kw-pad]           row stride ldc >= 9C
 *   dz[(b,y,x)][c] = sum_{kh,kw} dcols[(b,y-kh+pad,x-kw+pad)][c*9+kh*3+kw] * (a[b][c][y][x] > 0)
 * With them a conv layer's grads are GEMMs: dW = dz^T cols, db = colsum(dz),
 * dcols = dz W (then col2im for the layer below). */
int az_nchw_drelu_to_pm(const float* dy, const float* y, const uint8_t* mask, float scale,
                        int B, int C, int HW, float* dz, void* stream);
int az_im2col3x3(const void* in, int in_int8, int B, int C, int H, int W, int pad, int ldc,
                 float* cols, void* stream);
int az_col2im3x3_drelu(const float* dcols, int ldc, const float* a, int B, int C, int H, int W,
                       int pad, float* dz, void* stream);
/* GNNLayer backward (gnn_utils.py:34-74, per destination) from the activations the forward
 * kept in fwd_ws: writes dx [V][F] (input gradient) and every parameter gradient in `gr`.
 * The graph must carry the reverse CSR (src_rowptr/src_edges/dst_index). */
size_t az_gnn_layer_bwd_ws_bytes(int V, int E, int D, int F, int H);
int az_gnn_layer_bwd(const az_graph* g, const float* x, int F, int H, const az_gnn_layer_w* w,
                     const void* fwd_ws, const float* dout, float* dx,
                     const az_gnn_layer_grads* gr, void* ws, size_t ws_bytes, void* stream);
/* az_gnn_node_update_fwd's backward: from dout [V][F] and the forward's `save`:
 *   dx [V][F]   = dout on every row, + d/dx_d of the update on the destination rows;
 *   dagg [V][F] = d/dagg_d on the destination rows (other rows are not written);
 * and the six parameter gradients (written, same layout as the weights).
 * ws >= az_gnn_node_update_bwd_ws_bytes(D, F). */
size_t az_gnn_node_update_bwd_ws_bytes(int D, int F);
int az_gnn_node_update_bwd(const float* x, const float* agg, int V, int F, int D,
                           const int* dst_rows, const float* gate_w, const float* upd_w1,
                           const float* upd_w2, const float* save, const float* dout, float* dx,
                           float* dagg, float* d_gate_w, float* d_gate_b, float* d_upd_w1,
                           float* d_upd_b1, float* d_upd_w2, float* d_upd_b2, void* ws,
                           size_t ws_bytes, void* stream);
/* output_transform backward (gnn_utils.py:101-105): dW2, db2, dW0, db0, dh (scratch [M][F])
 * and dx (nullable).  ws >= az_colsum_ws_bytes(M, F) (+ split-K room). */
int az_mlp2_bwd(const float* x, int M, int F, const float* w0, const float* w2,
                const float* hidden, const float* dy, float* dx, float* dw0, float* db0,
                float* dw2, float* db2, float* dh, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * torch.optim.Adam step (defaults of Connect4GNN.py:132-133: betas (0.9,0.999), eps 1e-8,
 * no weight decay, no amsgrad) over one flat fp32 parameter buffer:
 *   m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
 *   p -= (lr / (1-b1^t)) m / (sqrt(v) / sqrt(1-b2^t) + eps)          (t = step >= 1)
 * --------------------------------------------------------------------------------- */
int az_adam_f32(float* p, const float* g, float* m, float* v, int64_t n,
                double lr, double beta1, double beta2, double eps, int step, void* stream);
/* The same call under SURVEY §8b's name (reference: torch.optim.Adam.step, Connect4GNN.py:187-197). */
int az_adam_step(float* p, const float* g, float* m, float* v, int64_t n,
                 double lr, double beta1, double beta2, double eps, int step, void* stream);

/* Parameters changed: every cached per-row weight scale and fp16 weight plane of the fp16 GEMM
 * form (az_gemm_f32's large K-major GEMMs on registered weights, below) is recomputed before its
 * next use.  The cache is keyed by the weight pointer and shape, so a caller that writes
 * registered weights any way other than az_adam_f32 (which calls it) -- an optimizer step of its
 * own, loading a checkpoint, copying buffers -- must call it before the next GEMM on them.
 * A missed call is NOT a precision loss: above 64 rows the GEMM multiplies by the cached planes,
 * i.e. it returns the PREVIOUS weights' result.  (azhip/params.py FlatParams calls it for the
 * torch-side writes that bump the buffer's version counter -- in-place ops on the parameter
 * tensors -- and from copy_flat_ / weights_changed().  Writes through `.data`, and collectives
 * that write parameter views in place (dist.broadcast / all_reduce), do not bump it: such a
 * path must call FlatParams.weights_changed() itself.) */
int az_weights_changed(void);

/* Parameter storage: [base, base + bytes) holds weights whose values change only where
 * az_weights_changed() says so.  Only weights inside a registered range have their fp16-form
 * row scales and pre-split planes cached (az_gemm_f32's large K-major GEMMs: W split once per
 * weight update instead of in every tile); any other weight pointer gets its scales computed per
 * call, since a pointer alone says nothing about the values behind it.  Registering or
 * unregistering also invalidates every cache entry; unregistering waits for the device and frees
 * the entries of weights inside the range (8 N K bytes each).  The Python parameter store
 * (azhip/params.py FlatParams) registers its flat buffer. */
int az_weights_register(const void* base, size_t bytes);
int az_weights_unregister(const void* base);

#ifdef __cplusplus
}
#endif
#endif /* AZ_HIP_H */
