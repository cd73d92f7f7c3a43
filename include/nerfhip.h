/*
 * nerfhip.h — C ABI of the MI355X (gfx950) NeRF volume-render library.
 *
 * Plain pointers and sizes only; every device pointer is HBM memory on the
 * current HIP device; every call takes an explicit stream (hipStream_t passed
 * as void*) and is asynchronous on it. Return value: 0 on success, otherwise
 * an error code (NERF_E_*) or a hipError_t; nerf_last_error() then holds a
 * message for the calling thread. Nothing here calls exit().
 *
 * Two groups of entry points:
 *   1. the render path of the reference PyTorch renderer
 *      (src/models/nerf/renderer/volume_renderer.py, "VR" below), split into
 *      the stages the reference runs per 2048-ray chunk;
 *   2. the op contract of the reference extension module `kilonerf_cuda`
 *      (cuda/pybind.cu:11-39), one kn_* function per op, same argument meaning.
 * Reference citations are file:line in the reference repository.
 */
#ifndef NERFHIP_H
#define NERFHIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* nerf_stream_t; /* hipStream_t */

enum {
  NERF_OK = 0,
  NERF_E_ARG = 1001,      /* bad argument (null pointer, size out of range) */
  NERF_E_UNSUPPORTED = 1002,
  NERF_E_LAUNCH = 1003,   /* kernel launch failed */
  NERF_E_HANDLE = 1004    /* unknown grouped-GEMM handle */
};

const char* nerf_last_error(void);
/* ABI version, bumped on every change of a struct layout or signature below
 * (2: NerfWgradDesc amax_a2/amax_b2/ldo, NerfX3BwdIO d_raw_t, the
 * nerf_sample_pdf_bwd / nerf_composite_ert arguments of round 4; 3: NerfWgradDesc
 * bsa / bsb, NerfX3TrainOut.bs / NerfX3BwdIO.bs and the encoding-backward layout
 * arguments: the T16 activation layout of round 5; 4: NerfWgradDesc.a2_row; 5: the
 * training forward's 65-slice (folded) stream, nerf_fold_views; 6: the backward's
 * 64-slice (folded) stream, NerfX3BwdIO.d[8] NULL; 7: nerf_views_feature_grads
 * GE / ldge) */
#define NERF_ABI_VERSION 7
int nerf_version(void);
/* 16 hex digits of sha256(the csrc/ files in byte order, then include/nerfhip.h): the
 * source tree this library was compiled from (nerfhip/_lib.py refuses a
 * library whose id differs from the tree beside it; the reference's
 * counterpart is its extension build, cuda/setup.py:13-24). */
const char* nerf_build_id(void);

/* ---------------------------------------------------------------------------
 * 1. Render path
 * ------------------------------------------------------------------------- */

/* Packed MLP layout: one 8x256 NeRF MLP = NERF_MLP_SLICES
 * slices of 32 KiB (MFMA A-fragments in consumption order) + a head block of
 * NERF_MLP_HEAD_FLOATS floats (lane-packed biases, density and rgb heads). */
#define NERF_MLP_SLICES 73
#define NERF_MLP_SLICE_FLOATS 8192
#define NERF_MLP_HEAD_FLOATS 3200
/* nerf_mlp_forward_x3's packing (nerfhip.pack.pack_mlp_x3) folds the
 * activation-free feature layer into the views layer: 65 slices. */
#define NERF_MLP_X3_SLICES 65

/* VR:115-143: camera rays for pixels [p0, p0+n) of an H x W image (row-major,
 * pixel p -> (y = p / W, x = p % W), integer pixel centres), origin = pose
 * translation, unit-length direction R·((x-cx)/fx, -(y-cy)/fy, -1) / |·|.
 * cam (device) = pose[16] (4x4 row-major) followed by K[9] (3x3 row-major).
 * rays_o, rays_d: [n][3] float32. */
int nerf_rays(const float* cam, int H, int W, int64_t p0, int64_t n,
              float* rays_o, float* rays_d, nerf_stream_t stream);

/* VR:218-237: coarse depths z[n][S]. z_base (device, [S]) is the reference's
 * torch.linspace-derived depth table; t_rand (device, [n][S], or NULL for
 * perturb = 0) the stratification draws. */
int nerf_sample_coarse(const float* z_base, const float* t_rand, int64_t n, int S,
                       float* z, nerf_stream_t stream);

/* NET:49-74 on samples pts = o + d*z of n rays x S samples (VR:165, VR:270-284):
 * frequency encoding (L=10 xyz, L=4 dir) fused with the 8x256 MLP, FP32 MFMA.
 * z row stride z_stride floats (0 = one shared row). raw: [n*S][4] = (rgb
 * logits, sigma raw). w_slices/w_head: packed by nerfhip.pack (device). */
int nerf_mlp_forward(const float* w_slices, const float* w_head,
                     const float* rays_o, const float* rays_d,
                     const float* z, int64_t z_stride, int64_t n, int S,
                     float* raw, nerf_stream_t stream);

/* Same contract as nerf_mlp_forward, computed with a 3-term FP16 split of the
 * FP32 operands on FP16 MFMA (w*x = wh*xh + wh*xl + wl*xh, exact products,
 * FP32 accumulation; power-of-two scaling keeps the splits in FP16 range):
 * ~2^-22 relative per product, 5.3x the FP32 MFMA arithmetic rate.
 * w_slices/w_head: packed by nerfhip.pack.pack_mlp_x3 (device). */
int nerf_mlp_forward_x3(const float* w_slices, const float* w_head,
                        const float* rays_o, const float* rays_d,
                        const float* z, int64_t z_stride, int64_t n, int S,
                        float* raw, nerf_stream_t stream);

/* Training-step compositing (VR:286-357, raw_noise_std 0), differentiable:
 * forward = the reference's maps for rays [n] with S samples (raw float4
 * [n*S], z [n][S], rays_d [n][3]) plus the weights and the exclusive
 * transmittance T [n][S] the backward reads; backward = d raw [n*S] (float4)
 * and, if d_z is not null, d z [n][S] from the gradients of any of the outputs
 * (null = zero). Replaces torch autograd's cumprod backward, whose host-side
 * zero test a HIP graph cannot capture (nerf-rep_for_test_amd/csrc/
 * train_kernels.hip). */
int nerf_composite_train_fwd(const float* raw, const float* z, const float* rays_d,
                             int64_t n, int S, int white, float* rgb, float* disp,
                             float* acc, float* depth, float* weights, float* trans,
                             nerf_stream_t stream);
int nerf_composite_train_bwd(const float* raw, const float* z, const float* rays_d,
                             const float* weights, const float* trans, const float* acc,
                             const float* depth, int64_t n, int S, int white,
                             const float* g_rgb, const float* g_disp, const float* g_acc,
                             const float* g_depth, const float* g_weights, float* d_raw,
                             float* d_z, nerf_stream_t stream);

/* Backward of _sample_fine with training-mode u (VR:239-268) + the merge
 * torch.sort(cat(z, z_fine)) (VR:181-184) whose forward is nerf_sample_fine:
 * d_weights [n][S] (rows 0 and S-1 zero) from g_zall [n][S + n_imp]. z [n][S],
 * weights [n][S], u [n][n_imp] as given to the forward; z_all [n][S + n_imp]
 * the forward's output (nullable: each fine sample's place in the merged row is
 * then counted instead of searched). S <= 130, n_imp <= 256. */
/* nerf_adam_step: one Adam step (torch.optim.Adam with weight_decay 0, no
 *   amsgrad; trainers/trainer.py's optimizer) over n <= 64 parameter tensors in
 *   ONE launch, each gradient first clamped in place to [-clip, clip]
 *   (clip_grad_value_, trainer.py:59; NaN kept; clip < 0: no clamp). tensors:
 *   host array {p, g, m (exp_avg), v (exp_avg_sq), n} (device float pointers).
 *   lr, step: device floats (the step count before this step; a second tiny
 *   launch on the stream leaves step + 1); done: unused (kept for the ABI,
 *   may be NULL). */
typedef struct NerfAdamTensor {
  float* p;
  float* g;
  float* m;
  float* v;
  int64_t n;
} NerfAdamTensor;
int nerf_adam_step(const NerfAdamTensor* tensors, int n, const float* lr, float* step,
                   unsigned* done, double beta1, double beta2, float eps, float clip,
                   nerf_stream_t stream);
/* nerf_fold_views (network.py:63-67): for each of n <= 4 networks, the views
 *   layer with the feature layer folded in, from the live parameters:
 *   Wc [128][283] = [W_views[:, :256] W_feat | W_views[:, 256:]] and
 *   bc [128] = W_views[:, :256] b_feat + b_views (FP32, k ascending) -- the
 *   views matrix and bias of the training forward's 65-slice stream. */
typedef struct NerfFoldDesc {
  const float* Wv;   /* views_linears.0.weight [128][283] */
  const float* Wf;   /* feature_linear.weight [256][256] */
  const float* bf;   /* feature_linear.bias [256] */
  const float* bv;   /* views_linears.0.bias [128] */
  float* Wc;         /* out [128][283] */
  float* bc;         /* out [128] */
} NerfFoldDesc;
int nerf_fold_views(const NerfFoldDesc* nets, int n, nerf_stream_t stream);
/* nerf_sum_partials: out[i] = sum_{c=0}^{C-1} part[c * n + i], summed in c
 *   order (the weight-gradient split-K partials of nerf_x3_wgrad). */
int nerf_sum_partials(const float* part, int64_t C, int64_t n, float* out, nerf_stream_t stream);
/* The views / feature / alpha weight gradients of the lego NeRF (NET:61-65)
 * from GA = [d_hv; d sigma] [h7; view enc]^T ([129][288+], row stride ldga) and
 * its row sums ba[129] (nerfhip.train_mlp): dWv [128][283] = [Gh W_f^T + s b_f^T,
 * GA[0:128, 256:283]], dWf [256][256] = W_v[:, :256]^T Gh, dbf [256] =
 * W_v[:, :256]^T s, dWa [256] = GA[128, 0:256], dba [1] = ba[128], dbv [128] =
 * s (Gh = GA[0:128, 0:256], s = ba[0:128]; W_f [256][256], b_f [256],
 * W_v [128][283] row-major). GE non-NULL (ABI 7): GE = [d_hv; d sigma; pad;
 * d rgb] [view enc; HV]^T ([147][160+], row stride ldge >= 160) and be its row
 * sums: the view-encoding columns come from GE[0:128, 0:27] instead of GA (GA
 * needs only its 256 h7 columns, ldga >= 256), and the rgb head's gradient is
 * copied out of it too: dWr [3][128] = GE[144:147, 32:160], dbr [3] =
 * be[144:147] (the training backward's shared tile, nerfhip.train_mlp). GE NULL:
 * be, dWr, dbr unused. */
int nerf_views_feature_grads(const float* GA, int64_t ldga, const float* ba, const float* Wf,
                             const float* bf, const float* Wv, float* dWv, float* dWf, float* dbf,
                             float* dWa, float* dba, float* dbv, const float* GE, int64_t ldge,
                             const float* be, float* dWr, float* dbr, nerf_stream_t stream);
/* trainers/nerf.py:39-76: out[0] = mean((a - target)^2), out[1] = the same of b
 * (0 when b is NULL), out[2] = out[0] + out[1] (a, b, target: N floats; one
 * workgroup). Backward: g0, g1, g2 = d out[0..2] (device scalars, each nullable
 * = 0); da = (2/N)(a - t)(g0 + g2), db = (2/N)(b - t)(g1 + g2). */
int nerf_mse_pair(const float* a, const float* b, const float* target, int64_t N, float* out,
                  nerf_stream_t stream);
int nerf_mse_pair_backward(const float* a, const float* b, const float* target, int64_t N,
                           const float* g0, const float* g1, const float* g2, float* da,
                           float* db, nerf_stream_t stream);
int nerf_sample_pdf_bwd(const float* z, const float* weights, const float* u,
                        const float* g_zall, const float* z_all, int64_t n, int S, int n_imp,
                        float* d_weights, nerf_stream_t stream);

/* ERT sample compaction (BASELINE configs[3]): nerf_mlp_forward_x3 over the
 * flat sample indices list[0 .. *count) (ray * S + step; count read on the
 * device, max_count bounds it), raw written at those indices. */
int nerf_mlp_forward_x3_list(const float* w_slices, const float* w_head,
                             const float* rays_o, const float* rays_d, const float* z,
                             int64_t z_stride, int S, const int* list, const int* count,
                             int64_t max_count, float* raw, nerf_stream_t stream);

/* One step of the segmented ERT evaluation: every ray with active[r] extends
 * its exclusive transmittance T[r] (double) over samples [s0, s1) from raw
 * with the ERT composite's alpha (VR:1091-1111); once T < thr (1 - 1e-6) it
 * is retired (its later samples are zero-weighted by _raw2outputs_with_ert,
 * VR:1115-1123), otherwise it appends the indices of its samples [s1, s2) to
 * list (slots from *count, atomically). */
int nerf_ert_segment(const float* raw, const float* z, int64_t z_stride, const float* rays_d,
                     int64_t n, int S, int s0, int s1, int s2, float thr, double* T,
                     unsigned char* active, int* list, int* count, nerf_stream_t stream);

/* Training MLP (BASELINE configs[2]): the 8x256 NeRF MLP of a training step
 * (network.py:49-74 forward and its autograd backward) as layer GEMMs over
 * feature-major activations ([F][P]: row f = feature f of every sample),
 * FP32 operands as 3-term FP16 splits on FP16 MFMA (see nerf_mlp_forward_x3).
 *
 * nerf_x3_layer: C[m][p] = 2^-(w_scale+e_p) * sum_k W[m][k] B[k][p]
 *   (+ bias[m]) (+ ru[m] * rw[p]) (ReLU if relu) (* (mask[m][p] > 0)),
 *   m < 16*m_tiles, k < 32*k_steps; W packed by nerfhip.train_mlp.pack_x3_matrix
 *   with its scale exponent in *w_scale (device int). The (shape, epilogue)
 *   instances are those the training MLP launches (nerf-rep_for_test_amd/csrc/
 *   mlp_x3.hip); others return NERF_E_UNSUPPORTED. amax_out (optional, device
 *   float, caller-initialised) is raised to max |C|.
 * nerf_x3_wgrad: part[c][m][n] = sum over the samples p of subset c of
 *   A[m][p] * B[n][p], for C = ceil(P / chunk) subsets (subset c = 32-sample
 *   steps c, c+C, c+2C, ...: their sum over c is the full product);
 *   amax_a / amax_b = device max|A|, max|B|; bias_part (optional) [c][m] =
 *   the same subsets' sums of A[m][p]. */
int nerf_x3_layer(const float* w_packed, const int* w_scale, int m_tiles, int k_steps,
                  const float* bias, const float* B, int64_t ldb, const float* mask,
                  int64_t ldm, const float* ru, const float* rw, int relu, float* C,
                  int64_t ldc, int64_t P, float* amax_out, nerf_stream_t stream);
/* nerf_x3_layer_ex: nerf_x3_layer with the ReLU mask carried as bits and an
 *   optional output head.
 *   relu_bits (nullable, needs relu) receives bit (C[m][p] > 0) of every output
 *   element; mask_bits (nullable, instead of mask) multiplies C by such a bit.
 *   Layout: u16 word ((p / 128 * 8 + p % 128 / 16) * m_tiles / 4 + m / 64) * 64
 *   + (p % 16) + 16 * (m % 16 / 4), bit 4 * (m % 64 / 16) + m % 4: the layer
 *   kernel's own lane order, so producer and consumer have the same m_tiles;
 *   ceil(P / 128) * 128 * m_tiles words. 32 B per sample and 256-wide layer,
 *   where the FP32 mask is 1 KiB.
 *   head_out (nullable): head_out[p * 4 + head_col + c] = sum_m head_w[c * 16 *
 *   m_tiles + m] * C[m][p] + head_b[c] for c < n_head (1..3, head_col + n_head
 *   <= 4; head_w 16-byte aligned): the alpha / rgb heads (network.py:61, 68-70)
 *   written straight into raw [P][4]. */
int nerf_x3_layer_ex(const float* w_packed, const int* w_scale, int m_tiles, int k_steps,
                     const float* bias, const float* B, int64_t ldb, const float* mask,
                     int64_t ldm, const float* ru, const float* rw, int relu, float* C,
                     int64_t ldc, int64_t P, float* amax_out, unsigned short* relu_bits,
                     const unsigned short* mask_bits, const float* head_w, const float* head_b,
                     int n_head, float* head_out, int head_col, nerf_stream_t stream);
int nerf_x3_wgrad(const float* A, int64_t lda, int M, const float* B, int64_t ldb, int N,
                  int64_t P, int64_t chunk, const float* amax_a, const float* amax_b,
                  float* part, float* bias_part, nerf_stream_t stream);
/* nerf_x3_wgrad_batch: n (<= 16) weight gradients of one backward in ONE
 *   launch, each split over `chunks` sample subsets (instead of ~256 per
 *   nerf_x3_wgrad call): subset c of descriptor k writes part + c * ldpart
 *   ([M][N]) and bias_part + c * ldbias ([M], optional); the same definitions
 *   as nerf_x3_wgrad. Operands must be aligned (P % 32 == 0, lda / ldb % 4 ==
 *   0, 16-byte aligned, < 2 GiB). descs is a host array (passed by value). */
typedef struct NerfWgradDesc {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  int64_t P;
  const float* amax_a;
  const float* amax_b;
  float* part;
  int64_t ldpart;
  float* bias_part;
  int64_t ldbias;
  int M, N;
  const float* amax_a2;   /* nullable: the A scale covers max(*amax_a, *amax_a2) */
  const float* amax_b2;   /* nullable: likewise for B */
  int64_t ldo;            /* row stride of the partials ([M][ldo] at part + z * ldpart);
                             0: N. Two descriptors with the same A can write the column
                             blocks of one gradient (the skip layer's [enc | h4]) */
  int64_t bsa, bsb;       /* sample-block strides of A / B in floats (ABI 3): element (r, p)
                             of an operand is at r * ld + (p / 16) * bs + p % 16. 0 (or 16):
                             feature-major rows ([M][ld], ld >= P); 16 * rows with ld = 16:
                             the 16-sample block layout [P / 16][rows][16] of the fused
                             training kernels (nerf_mlp_train_forward_x3) */
  int a2_row;             /* (ABI 4) 0: amax_a2 widens the one A scale, as above. > 0 (a
                             multiple of 16, < M, amax_a2 set): rows < a2_row of A take
                             the scale of *amax_a, rows >= a2_row that of *amax_a2 -- two
                             row blocks of one operand with their own FP16 split ranges */
} NerfWgradDesc;
int nerf_x3_wgrad_batch(const NerfWgradDesc* descs, int n, int chunks, nerf_stream_t stream);
/* The same with a K split per output tile: tile_chunks[t] (1 .. zmax, < 256)
 *   for the tiles in the order descriptor, N tile, M tile (256 x 256 tiles, at
 *   most 40); subset c < tile_chunks[t] of tile t writes partial row c, rows
 *   tile_chunks[t] .. zmax-1 of the tile (and of its bias rows) are zeros. */
int nerf_x3_wgrad_batch_z(const NerfWgradDesc* descs, int n, const int* tile_chunks, int zmax,
                          nerf_stream_t stream);

/* nerf_mlp_train_forward_x3: the whole forward of a training step's MLP in ONE
 *   launch (the inference kernel over the 65-slice stream, the feature layer
 *   folded into the views layer (ABI 5): nerfhip.pack.pack_mlp_x3, or its
 *   device-side packer nerfhip.train_mlp.X3StreamPacker after nerf_fold_views).
 *   Samples p = 0 .. P-1 at pts[p]
 *   ([P][3]) with view direction dirs[p]; `zero` = one device float 0.0.
 *   raw[p] = (rgb logits, sigma) as nerf_mlp_forward_x3; besides, every
 *   output is written feature-major with row stride out->ld floats:
 *   act[L] = h_L (rows 0..255) for L = 0..7, act[8]: unused (NULL; the feature
 *   rows are not computed),
 *   act[9] = the views layer's output (128 rows), act[10] = the xyz encoding
 *   (64 rows: freq.py's 63 columns, row 63 = 0), act[11] = the view encoding
 *   (32 rows: 27 columns, rows 27..31 = 0); bits[L] = the ReLU bits of h_L
 *   (nerf_x3_layer_ex's layout, m_tiles 16) for L = 0..7 and bits[8] those of
 *   the views output (m_tiles 8); amax[0..11] (device floats,
 *   caller-initialised, >= 0) are raised to max |h_0..h_7|, (slot 8 untouched),
 *   max |xyz encoding|, max |view encoding|, max |views output|. The weight
 *   gradients of the views and feature layers are taken through h_7
 *   (nerfhip.train_mlp: dW_views,feat = G W_feat^T + s b_feat^T with
 *   G = d_hv h_7^T). */
typedef struct NerfX3TrainOut {
  float* act[12];
  unsigned short* bits[9];
  float* amax;
  int64_t ld;
  int64_t bs;   /* 0: feature-major rows (row stride ld >= P); > 0 (a multiple of 256):
                   the T16 layout, block stride bs floats, every act[] a row of one
                   [ceil(P/128) * 8][rows][16] buffer starting on a 16-row group:
                   row 16 t + 4 g + r of sample 16 b + s at b * bs + t * 256 + r * 64 +
                   g * 16 + s (ABI 3; nerfhip.train_mlp.BlockRows) */
} NerfX3TrainOut;
int nerf_mlp_train_forward_x3(const float* w_slices, const float* w_head, const float* pts,
                              const float* dirs, const float* zero, int64_t P,
                              const NerfX3TrainOut* out, float* raw, nerf_stream_t stream);
/* The same over the samples of n rays (VR:165): sample p = ray * S + step at
 * rays_o[ray] + rays_d[ray] * z[ray * z_stride + step], view direction
 * rays_d[ray]; P = n * S (the point tensor and the per-sample directions are
 * never materialised). */
int nerf_mlp_train_forward_x3_rays(const float* w_slices, const float* w_head,
                                   const float* rays_o, const float* rays_d, const float* z,
                                   int64_t z_stride, int64_t n, int S, const NerfX3TrainOut* out,
                                   float* raw, nerf_stream_t stream);

/* nerf_mlp_train_backward_x3: the backward through the training MLP (the
 *   dgrad chain) in ONE launch, over the transposed-weight stream of
 *   nerfhip.train_mlp.X3BwdStreamPacker (64 slices with_enc, 60 without; the
 *   feature layer folded into the views layer as in the forward: its first
 *   4 slices are Wc[:, :256]^T of nerf_fold_views, ABI 6).
 *   From io->d_raw ([P][4]: d rgb logits, d sigma; 16-byte aligned) and the
 *   forward's ReLU bits (io->bits as NerfX3TrainOut.bits), writes with row
 *   stride io->ld: d[9] = d_hv (128 rows), d[7] .. d[0] = the gradients of
 *   the pre-activations of layers 7 .. 0 (256 rows each); with_enc also
 *   d[10] / d[11] = the xyz encoding's gradient through layer 5 / layer 0
 *   (64 rows; row 63 is padding). d[8] must be NULL: d feature does not exist
 *   (dW_feat = W_views,feat^T G, see NerfX3TrainOut). io->dmax[0..7], [10]
 *   (caller-initialised, >= 0) are raised to the outputs' max |.|, [11] / [12]
 *   to max |d rgb| / |d sigma| of d_raw; [8] is untouched. */
typedef struct NerfX3BwdIO {
  const float* d_raw;
  const unsigned short* bits[9];
  float* d[12];
  float* dmax;
  int64_t ld;
  float* d_raw_t;   /* nullable: d raw as rows: d sigma at row 0, d r, d g, d b at rows 1..3
                       (feature-major, stride ld) or 16..18 (T16: a 16-row group of their own) */
  int64_t bs;       /* as NerfX3TrainOut.bs (ABI 3) */
} NerfX3BwdIO;
/* nerf_mlp_forward_x3_clock: nerf_mlp_forward_x3's computation (same outputs)
 *   by a diagnostic twin of its kernel that stamps (s_memtime, s_memrealtime)
 *   around each workgroup's work: clk[4 b + 0..3] = (memtime start, end,
 *   realtime start, end) of workgroup b (clk 32-byte aligned, clk_len >= 4 x
 *   workgroups; entries past the launched workgroups are left as they were).
 *   The held shader clock = d memtime / d realtime x 100 MHz. trace (512 x 4
 *   u64): workgroups 0..3 stamp memtime at each of their first 32 tiles'
 *   start, after its sample loads + encoding, and at its end:
 *   trace[(b * 32 + i) * 4 + 0..2]. */
int nerf_mlp_forward_x3_clock(const float* w_slices, const float* w_head, const float* rays_o,
                              const float* rays_d, const float* z, int64_t z_stride, int64_t n,
                              int S, float* raw, unsigned long long* clk, int64_t clk_len,
                              unsigned long long* trace, nerf_stream_t stream);
int nerf_mlp_train_backward_x3(const float* w_slices, const float* w_head, int64_t P,
                               int with_enc, const NerfX3BwdIO* io, nerf_stream_t stream);
/* nerf_raw_absmax: amax[0] / amax[1] (caller-initialised, >= 0) raised to
 *   max |raw[p][0..2]| / max |raw[p][3]| over p < P (the rgb / alpha heads'
 *   weight-gradient scales from d_raw [P][4], 16-byte aligned). */
int nerf_raw_absmax(const float* raw, int64_t P, float* amax, nerf_stream_t stream);
/* nerf_freq_encode_fm: the frequency encoding of freq.py:7-32 (reference
 *   embed_fn / embeddirs_fn, encoding/__init__.py:7-18), written feature-major
 *   for the training MLP: out[j * ldo + p] for the 3 + 6 * n_freq columns of
 *   torch.cat([x, sin(2^0 x), cos(2^0 x), ...], -1) of sample p (x [P][ldx],
 *   3 coordinates). amax (nullable, device float >= 0) is raised to the
 *   largest |out| (atomic max). */
int nerf_freq_encode_fm(const float* x, int64_t ldx, int64_t P, int n_freq, float* out,
                        int64_t ldo, float* amax, nerf_stream_t stream);
/* nerf_freq_encode_fm_backward: dx [P][3] = d(encoding)/dx^T d_enc, d_enc
 *   feature-major [3 + 6 * n_freq][ldd]. */
int nerf_freq_encode_fm_backward(const float* d_enc, int64_t ldd, const float* x, int64_t ldx,
                                 int64_t P, int n_freq, float* dx, nerf_stream_t stream);
/* The same on d_enc + d_enc2 (elementwise, same layout; d_enc2 nullable): the
 * encoding's two consumers' gradients summed in the kernel. enc (nullable):
 * the forward's encoding rows, whose sin / cos values are read instead of
 * recomputed. Layouts (ABI 3): d_enc / d_enc2 (ldd, bsd), enc (lde, bse); bs 0 =
 * feature-major rows of stride ld (>= P), bs > 0 = the T16 layout of
 * NerfX3TrainOut.bs. */
int nerf_freq_encode_fm_backward_sum(const float* d_enc, const float* d_enc2, int64_t ldd,
                                     int64_t bsd, const float* enc, int64_t lde, int64_t bse,
                                     const float* x, int64_t ldx, int64_t P, int n_freq,
                                     float* dx, nerf_stream_t stream);
/* ... taken on to the sample depths of nerf_mlp_train_forward_x3_rays: dz[p] =
 * sum_c dx[p][c] * rays_d[p / S][c] (enc required). */
int nerf_freq_encode_fm_backward_dz(const float* d_enc, const float* d_enc2, int64_t ldd,
                                    int64_t bsd, const float* enc, int64_t lde, int64_t bse,
                                    const float* rays_d, int S, int64_t P, int n_freq, float* dz,
                                    nerf_stream_t stream);
/* nerf_x3_pack: packs n weight matrices for the x3 training kernels in one
 * launch set. descs (device) = n records {const float* src; int64_t ldr, ldc;
 * const int* rowmap; const int* colmap; int M, K; void* out; int* sw;
 * unsigned* amax} (72 bytes each): padded element (i, k) = src[rowmap[i]*ldr +
 * colmap[k]*ldc] (0 where a map entry is -1); out receives the FP16 (hi, lo)
 * fragments, *sw the scale exponent; *amax must be 0 on entry and is 0 again
 * on exit. heads (device) = n_heads records {const uint64_t* table; float* dst;
 * int64_t n}: dst[i] = the float at address table[i], or (bit 0 set) the scale
 * exponent of the matrix whose amax slot is table[i] - 1, or 0 (table[i] 0). */
int nerf_x3_pack(const void* descs, int n, const void* heads, int n_heads, nerf_stream_t stream);

/* NET:9-74 for network topologies other than lego's (the fused MLP kernels'
 * one): one nn.Linear (+ ReLU when relu != 0) in FP32 over feature-major
 * activations, Y[m * sym + p * syp] = act(b[m] + sum_k W[m * ldw + k] X[k * ldx + p])
 * for m < M, p < P; b nullable; the k sum in ascending order. Used layer by
 * layer by nerfhip.generic_mlp, and for the training forward's per-step fold of
 * the feature layer into the views layer (W_views,feat W_feat). */
int nerf_linear_fm(const float* W, int64_t ldw, const float* b, const float* X, int64_t ldx,
                   int K, int64_t P, int M, int relu, float* Y, int64_t sym, int64_t syp,
                   nerf_stream_t stream);

/* VR:310-314, :1098-1103 (raw_noise_std > 0): out[i] = raw[i] with its density
 * logit (.w) plus noise[i] -- the caller's torch.randn(...) * raw_noise_std in the
 * reference's draw order; raw / out float4 [count], noise [count]; out may be
 * raw. The composites then read out (the ESS grid update keeps the raw without
 * noise, as VR:1150-1153 does). */
int nerf_add_sigma_noise(const float* raw, const float* noise, int64_t count, float* out,
                         nerf_stream_t stream);

/* VR:286-357: alpha compositing of raw[n*S][4] along z (row stride z_stride).
 * Reductions follow torch's CPU float32 summation order.
 * Outputs rgb[n][3], disp/acc/depth[n]; weights[n][S] optional (NULL). */
int nerf_composite(const float* raw, const float* z, int64_t z_stride,
                   const float* rays_d, int64_t n, int S, int white_bkgd,
                   float* rgb, float* disp, float* acc, float* depth, float* weights,
                   nerf_stream_t stream);

/* VR:1089-1133: compositing with early ray termination, including the
 * chunk-wide argmax behaviour: rays are grouped in chunks of `chunk` rays
 * (2048 in the reference, VR:147) counted from ray 0 of this call.
 * workspace: device memory of nerf_composite_ert_workspace(n, chunk) bytes
 * (16-B aligned; the per-ray cut maps and the per-chunk decisions of the
 * two-pass implementation), owned by the caller, one call at a time. */
size_t nerf_composite_ert_workspace(int64_t n, int chunk);
int nerf_composite_ert(const float* raw, const float* z, int64_t z_stride,
                       const float* rays_d, int64_t n, int S, int white_bkgd,
                       float threshold, int chunk,
                       float* rgb, float* disp, float* acc, float* depth, float* weights,
                       void* workspace, nerf_stream_t stream);

/* VR:239-268 + VR:181-183: inverse-CDF fine sampling from the coarse weights
 * and merge: z_all[n][S+n_imp] = sort(concat(z, samples)).
 * u: [n_imp] (u_stride 0, eval) or [n][n_imp] (training draws).
 * Limits: 3 <= S <= 130 coarse samples, 1 <= n_imp <= 256. */
int nerf_sample_fine(const float* z, int64_t z_stride, const float* weights,
                     const float* u, int64_t u_stride, int64_t n, int S, int n_imp,
                     float* z_all, nerf_stream_t stream);

/* VR:1009-1087 empty-space skipping for whole chunks of `chunk` rays: per
 * chunk one shared depth row folded over its "highly empty" rays in ray order
 * (the reference's expand()-shared row), then optional stratification.
 * grid: bool[res^3] (x-major, [x][y][z]) over the box [-2,2]^3. S <= 64. */
int nerf_sample_coarse_ess(const float* rays_o, const float* rays_d,
                           const uint8_t* grid, int res, const float* z_base,
                           const float* t_rand, int64_t n, int S, int chunk,
                           float skip_threshold, float* z, nerf_stream_t stream);

/* VR:1147-1155 / VR:963-990: occupancy-grid self-update: cells of points
 * d*z (no origin, as the reference) with weight > 1e-4 and relu(sigma) > 0.01
 * are set. */
int nerf_grid_update(const float* rays_d, const float* z, int64_t z_stride,
                     const float* raw, const float* weights, int64_t n, int S,
                     uint8_t* grid, int res, nerf_stream_t stream);

/* VR:875-961 (_populate_occupancy_grid_kilonerf_method), in two launches
 * around the MLP: nerf_grid_points writes the 27 sub-points of cells
 * [cell0, cell0 + ncells) (cell f: x = f % res, y = (f % res^2) / res,
 * z = f / res^2; sub-point 9 dz + 3 dy + dx at bbox_min + (x, y, z) * cell +
 * (dx, dy, dz) / 2 * cell, torch's float32 op order) into pts[ncells * 27][3];
 * the caller evaluates the coarse MLP on them (raw[ncells * 27][4]);
 * nerf_grid_decide sets grid[cell_of[f]] (or, cell_of NULL, the cell's own
 * [x][y][z] index) for every cell whose max relu(sigma) exceeds threshold
 * (0.01 in the reference). bbox_min / cell_size: host arrays. The caller
 * zeroes the grid first (VR:894). */
int nerf_grid_points(int64_t cell0, int64_t ncells, int res, const float bbox_min[3],
                     const float cell_size[3], float* pts, nerf_stream_t stream);
int nerf_grid_decide(const float* raw, int64_t cell0, int64_t ncells, int res, float threshold,
                     const int32_t* cell_of, uint8_t* grid, nerf_stream_t stream);

/* ---------------------------------------------------------------------------
 * 2. kilonerf_cuda op contract (cuda/pybind.cu:13-38)
 * ------------------------------------------------------------------------- */

/* cuda/generate_inputs.cu:11-52 — un-normalised R·((x-cx)/fx, -(y-cy)/fy, -1),
 * out [H][W][3]; c2w (device) 3x3 row-major. */
int kn_get_rays_d(int H, int W, float cx, float cy, float fx, float fy,
                  const float* c2w, float* out, nerf_stream_t stream);

/* cuda/generate_inputs.cu:60-192 */
int kn_generate_query_indices_on_ray(const float* origin, const float* directions, int num_rays,
                                     const int16_t* occupancy_grid, uint8_t* active_ray_mask,
                                     int16_t* depth_indices, const float* voxel_size,
                                     const float* global_domain_min, const float* global_domain_max,
                                     const int32_t* strides, float distance_between_points,
                                     int max_samples_per_ray, int max_depth_index,
                                     float min_distance, int is_initial_query,
                                     int32_t* query_indices, int16_t* assigned_networks,
                                     nerf_stream_t stream);

/* cuda/fourier_features.cu:8-100 — per scalar [x, cos(f_0 x)..cos(f_{L-1}x),
 * sin(f_0 x)..sin(f_{L-1}x)], out [n*(2L+1)]. */
int kn_compute_fourier_features(const float* input, int64_t n, const float* freqs, int L,
                                float* out, nerf_stream_t stream);

/* cuda/integrate.cu:9-81 — post-activation rgb_sigma [num_rays*spr][4],
 * per-ray dists [num_rays]; rgb_map [num_rays][3] (the reference passes it as
 * a raw int64 address), acc/T/mask in place. */
int kn_integrate(const float* rgb_sigma, const float* dists, float* rgb_map, float* acc_map,
                 float* transmittance, uint8_t* active_ray_mask, int num_rays,
                 int samples_per_ray, float transmittance_threshold, int is_initial_query,
                 nerf_stream_t stream);

/* cuda/integrate.cu:83-112 — rgb += bg * (1 - acc), n pixels. */
int kn_replace_transparency_by_background_color(float* rgb_map, const float* acc_map, int64_t n,
                                                const float* background_color /* device [3] */,
                                                nerf_stream_t stream);

/* cuda/reorder.cu:13-49 */
int kn_gather_int32(const int32_t* map, int64_t n_out, const int32_t* input, int32_t* out,
                    nerf_stream_t stream);
int kn_scatter_int32_float4(const int32_t* map, int64_t n, const float* input /*[n][4]*/,
                            float* out /*[..][4]*/, nerf_stream_t stream);
/* stable sort of (key, value) pairs by int16 key, in place; scratch: device
 * bytes >= kn_sort_scratch_bytes(n, value_bytes). value_bytes = 4 or 8. */
size_t kn_sort_scratch_bytes(int64_t n, int value_bytes);
int kn_sort_by_key_int16(int16_t* keys, void* values, int value_bytes, int64_t n,
                         void* scratch, nerf_stream_t stream);

/* cuda/global_to_local.cu:8-62 — in place p = 2(p-min_k)/(max_k-min_k)-1 per
 * network segment; batch_size_per_network is HOST memory (the reference reads
 * it on the host, global_to_local.cu:36-47). */
int kn_global_to_local(float* points, const float* domain_mins, const float* domain_maxs,
                       const int64_t* batch_size_per_network_host, int num_networks,
                       nerf_stream_t stream);

/* cuda/network_eval.cu:24-297 — KiloNeRF tiny-MLP evaluation (hidden 32). */
int kn_network_eval_query_index(const int32_t* query_indices, int64_t batch, const float* params,
                                const float* domain_mins, const float* domain_maxs,
                                const int32_t* starts, const int32_t* ends,
                                const float* origin, const float* c2w, int num_networks,
                                int hidden_dim, int H, int W, float cx, float cy, float fx,
                                float fy, int max_depth_index, float min_distance,
                                float distance_between_samples, float* out /*[batch][4]*/,
                                nerf_stream_t stream);

/* cuda/multimatmul.cu:18-100 — stream pool and MAGMA init (MAGMA is not used:
 * the grouped GEMM is a native kernel; init_magma succeeds as a no-op). */
int kn_init_stream_pool(int64_t num_streams);
int kn_destroy_stream_pool(void);
int kn_init_magma(void);

/* cuda/multimatmul.cu:152-428 — grouped GEMM over consecutive row segments:
 * for network k with b_k rows, out[rows_k][out_f] = X[rows_k][in_f] · op(W_k)
 * (+ bias_k). The reference's MAGMA column-major views mean
 *   mode 0 (static, with bias) / 1 (without bias): W_k stored [in_f][out_f];
 *   mode 2 (without bias, transposed weights):     W_k stored [out_f][in_f].
 * bias: [num_networks][out_f] (mode 0 only). batch_size_per_network is HOST
 * memory (the reference reads it on the host). Handle = returned by init; it
 * owns a device buffer of num_networks + 1 row offsets, rewritten by each call
 * (stream-ordered), so one handle serves one stream at a time, as the
 * reference's per-handle MAGMA state does. deinit synchronises the device
 * before freeing it. */
int kn_init_multimatmul_grouped(int64_t num_networks, int64_t out_features, int64_t in_features,
                                const int32_t* group_limits, int n_group_limits, int* handle);
int kn_deinit_multimatmul_grouped(int handle);
int kn_multimatmul_grouped(int handle, int mode, const float* biases, const float* X,
                           const float* W, int64_t out_features, int64_t in_features,
                           const int64_t* batch_size_per_network_host, int num_networks,
                           float* out, nerf_stream_t stream);

/* cuda/multimatmul.cu:430-524 — per-network column sums of M [Σb][cols]. */
int kn_multi_row_sum_reduction(const float* M, int64_t cols,
                               const int64_t* batch_size_per_network_host, int num_networks,
                               float* out /*[num_networks][cols]*/, nerf_stream_t stream);

/* cuda/multimatmul.cu:527-623 — per-network A_k^T · B_k, A [Σb][a_cols],
 * B [Σb][b_cols] -> out [num_networks][a_cols][b_cols]. */
int kn_multimatmul_A_transposed(const float* A, int64_t a_cols, const float* B, int64_t b_cols,
                                const int64_t* batch_size_per_network_host, int num_networks,
                                float* out, nerf_stream_t stream);

/* cuda/render_to_screen.cpp:222-248 — OpenGL viewer: not supported. */
int kn_render_to_screen(void);

#ifdef __cplusplus
}
#endif
#endif /* NERFHIP_H */
