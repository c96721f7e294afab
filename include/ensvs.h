/*
 * ensvs.h — C ABI of libensvs.so, the MI355X (gfx950) kernels behind the
 * multi-track ensemble SVS acoustic-model path.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t
 * (passed as void*), never allocates, never synchronises the host, and
 * returns 0 on success or an ENSVS_E_* code.  All activation tensors are
 * fp32, channels-last frame rows: element (b, t, c) at base + (b*T + t)*ld + c.
 *
 * Each entry point names the reference code it replaces
 * (paths relative to sarulab-speech/ensemble_svs_with_interactions).
 */
#ifndef ENSVS_H_
#define ENSVS_H_

#ifdef __cplusplus
extern "C" {
#endif

enum { ENSVS_STATUS_OK = 0, ENSVS_STATUS_E_SHAPE = 1, ENSVS_STATUS_E_DTYPE = 2,
       ENSVS_STATUS_E_HIP = 3, ENSVS_STATUS_E_ARG = 4 };
enum { ENSVS_PAD_ZERO = 0, ENSVS_PAD_REFLECT = 1, ENSVS_PAD_REPLICATE = 2 };
enum { ENSVS_DT_F32 = 0, ENSVS_DT_BF16 = 1 };
enum { ENSVS_EPI_PLAIN = 0, ENSVS_EPI_GATE = 1, ENSVS_EPI_RESSKIP = 2, ENSVS_EPI_GATE_BWD = 3,
       ENSVS_EPI_ADDSCALE = 4, ENSVS_EPI_RELU_MASK = 5, ENSVS_EPI_GATE_TS = 6,
       /* flags or-ed into `epi`: the DiffNet gate/filter save in bf16 (GATE writes aux0,
        * GATE_BWD reads aux1 as bf16 rows; the production bf16 path) */
       ENSVS_EPI_AUX0_BF16 = 256, ENSVS_EPI_AUX1_BF16 = 512 };

/* One K-segment of the implicit-GEMM activation operand. */
typedef struct ensvs_conv_seg {
  const float* x;     /* frame rows (offset to the segment's first channel) */
  const float* radd;  /* optional per-sequence vector added to in-range values */
  const float* pd;    /* optional (first segment, taps 3): per-row pitch-dependent dilation
                         factor; taps become past / current / future samples gathered with
                         the uSFGAN index arithmetic (usfgan/utils/index.py:12-54) */
  long long wofs;     /* element offset of packed weights [taps][Npad][Kp] */
  int ld, K, taps, dil, shift0, pad, radd_ld, Tin, Kp;
  int pd_dil;         /* dilation multiplying pd */
} ensvs_conv_seg;

/* Weight repack descriptor (reference layout -> GEMM layout [tap][Npad][Kp]). */
typedef struct ensvs_pack_desc {
  const float* src;
  const float* src2;
  void* dst;
  long long sn, sk, sj;
  int N, K, taps, Npad, Kp, perm_c, flip, transpose, dtype;
  float scale;
  int ldk;    /* destination row stride in elements (0: Kp) */
  int tile0;  /* ensvs_pack_weights_tiled: the descriptor's first tile (ignored otherwise) */
} ensvs_pack_desc;

/* Conv1d / Linear forward and input-gradient as an MFMA implicit GEMM.
 * Replaces nn.Conv1d / nn.Linear / nn.ReflectionPad1d call sites in
 * nnsvs/model.py:837-859 (FFConvLSTM.ff/.conv), nnsvs/acoustic_models/tacotron_f0.py:852-874,
 * the DiffNet convolutions nnsvs/diffsinger/denoiser.py:40-66,101-124 and every uSFGAN
 * generator convolution (usfgan/layers/residual_block.py:123-234,389-399, upsample.py:166-168,
 * usfgan/models/generator.py:427-466).  `relu`: output activation of EPI_PLAIN / EPI_ADDSCALE
 * (1 ReLU, 2 sigmoid). */
int ensvs_conv_gemm(const ensvs_conv_seg* segs, int nseg, int B, int Tout, int N, int Npad,
                    const void* W, int wdtype, const float* bias, float* Y, int ldy, int epi,
                    int relu, int accum, float* aux0, int ld0, const float* aux1, int ld1,
                    float alpha, int C, void* stream);

/* The same contraction with bf16 activations: every segment's x is a const __bf16* (ld and
 * K multiples of 8, 16-B aligned, radd and pd NULL) -- ensvs_cast_bf16 output, which
 * holds the rounding ensvs_conv_gemm applies while staging, so both give identical bits.
 * Operands are staged by global_load_lds, `stages` (2 or 3) 64-deep K tiles.  wdtype is bf16. */
/* Large-M bf16-operand launches (>= 192 tiles of 256 x 256, padded N % 256 == 0, no column
 * sums) run a 256 x 256-tile kernel with the same accumulation order (bitwise equal).
 * mode 0: keep the 128 x 128 kernel; 1: 32-deep K steps on a `stages`-deep LDS ring
 * (3..5; 0 keeps the current count); 2: 64-deep two-stage kernel for the gate GEMMs (the
 * other epilogues run faster on 128 x 128 tiles); 3: as 2 for every eligible launch.
 * Defaults: mode 2, 5 stages. */
int ensvs_set_big_tile(int mode, int stages);
/* The four-phase 256 x 256 kernel (counted LDS-DMA pipeline, four half-tiles in flight across
 * every barrier; same accumulation order, bitwise equal): mode & 3 -- 0 off; 1 for the launches
 * the 256 x 256 kernel takes (gate GEMMs); 2 also for every other launch its LDS-staged
 * epilogue serves with >= 128 tiles of 256 x 256 (no column sums, not the LDS-DMA epilogues);
 * 3 the gate GEMMs and the lean plain launches only; + 4: two barriers per phase with the wave
 * rows staggered half a phase (without: one barrier per phase, rows in lockstep); default 6;
 * + 8 / + 16: measurement only -- EPI_NONE launches run the K loop without its operand loads /
 * without its MFMAs (what each costs). */
int ensvs_set_p8(int mode);
/* The four-phase kernel's smallest launch for its non-gate epilogues, in tiles of 256 x 256
 * (default 128; A/B). */
int ensvs_set_p8_min_tiles(int n);
/* The 128 x 256 kernel (the four-phase pipeline on half-height tiles, two phases per K-step,
 * three K-step buffers) for launches the 256 x 256 kernel leaves with < 128 tiles: mode 0 off;
 * 1 (default) the plain epilogues (lean or with operands, copies, column sums) and ADDSCALE /
 * RELU_MASK without column sums (where it beats the 128 x 128 kernel); 2 every launch but the pair
 * epilogues (gate, res/skip), column sums included (A/B, tests); 3 the lean plain launches only;
 * + 4 k: modes 1 / 3 only for launches of >= k K-steps (default k = 1).  Same accumulation and
 * column-sum order: bitwise equal. */
int ensvs_set_p8h(int mode);
/* Launches of fewer than 128 output tiles (small M) that the 64 x 64 kernel does not take
 * can run a 128 x 128 kernel with two K-groups of 4 waves (each group half of the K-steps,
 * tiles added through LDS; default off: the one-group kernel, the same bits as the
 * register-staged kernel; kept for the sum-order tests). */
int ensvs_set_dual_small(int on);
/* Both LDS-DMA epilogues -- the DiffNet gate-backward dgrad (EPI_GATE_BWD, production form)
 * and the dilated-conv dgrad's ADDSCALE epilogue -- (default 1) or their register-batched
 * forms (0): same bits; for the bitwise tests.  One switch covers both. */
int ensvs_set_gbw_dma(int on);
/* bf16-operand weight gradients with N, K >= 256 on the 256 x 256-tile kernel (default 1) or
 * the 128 x 128 one (0): same bits for the same split count. */
int ensvs_set_wgrad_big(int on);
/* Launches of fewer than 128 output tiles of 128 x 128 (small M: the 2 000-frame reverse-
 * diffusion GEMMs) run a 64 x 64-tile kernel that fills the chip (default on; it takes
 * precedence over the two-K-group kernel and split-K); same accumulation order as the
 * one-group kernel, so the same bits.  0 turns it off; 2 (A/B) also gives it the N <= 128
 * launches of < 256 tiles of 128 x 128 (one workgroup per CU on the 128 x 128 kernel). */
int ensvs_set_small(int on);
/* Persistent recurrence workgroups (LSTM, AR decoder) reserve their CU's LDS so no GEMM
 * workgroup of a concurrent stream lands beside them (default on);
 * read at each launch, so a caller can choose per branch. */
int ensvs_set_recurrence_exclusive(int on);
/* One uSFGAN residual block in one launch (usfgan/layers/residual_block.py): the gate GEMM
 * over bf16 segments (x's copy with taps 3 / optional pd, the aux features' copy; packed
 * gate/filter columns interleaved by 16, 2C = 128), z = tanh(gate) * sigmoid(filter) kept on
 * chip in bf16, the 1x1 output conv (packed at wofs2, Kp2 = 64) and
 * x = alpha * x + out + bias2 (ReLU when relu) in place, with x's bf16 copy in xb (optional).
 * C = 64.  Same bits as the gate GEMM with a bf16 z copy followed by the output GEMM. */
int ensvs_usf_block(const ensvs_conv_seg* segs, int nseg, int B, int Tout, const void* W,
                    const float* bias1, int C, long long wofs2, int Kp2, const float* bias2,
                    float* x, int ldx, float alpha, int relu, void* xb, int xb_ld, void* stream);
/* part / part_floats (optional, may be NULL / 0): fp32 workspace for split-K.  Launches of
 * fewer than 128 output tiles (small M: the 2 000-frame reverse-diffusion GEMMs) split their
 * K-steps over up to 8 workgroups per tile when part holds ksplit x M x Npad floats; the
 * slices are summed in a fixed order by a second kernel that runs the epilogue
 * (deterministic; the Python wrapper passes no workspace by default).  Operand rows: bf16, ld % 8 == 0, 16-B aligned;
 * a segment with K % 8 != 0 has its rows zero-padded to a multiple of 8 within ld. */
int ensvs_conv_gemm_bf16a(const ensvs_conv_seg* segs, int nseg, int B, int Tout, int N, int Npad,
                          const void* W, const float* bias, float* Y, int ldy, int epi, int relu,
                          int accum, float* aux0, int ld0, const float* aux1, int ld1, float alpha,
                          int C, int stages, float* part, long long part_floats, void* stream);
/* ensvs_conv_gemm_bf16a that also writes ybf[row*ybf_ld + col] = bf16(y + ybf_radd[(row /
 * Tout)*ybf_radd_ld + col]) for every output it writes (the next GEMM's operand, rounded as
 * ensvs_cast_bf16 would, without that pass).  Needs 16-B output rows (ld % 4 == 0) and
 * N % 4 == 0; returns ENSVS_E_ARG otherwise. */
int ensvs_conv_gemm_bf16a_out(const ensvs_conv_seg* segs, int nseg, int B, int Tout, int N,
                              int Npad, const void* W, const float* bias, float* Y, int ldy,
                              int epi, int relu, int accum, float* aux0, int ld0,
                              const float* aux1, int ld1, float alpha, int C, void* ybf,
                              int ybf_ld, const float* ybf_radd, int ybf_radd_ld, float* csum,
                              int csum_ld, int stages, float* part, long long part_floats,
                              void* stream);
/* csum (optional, M % 128 == 0): per 128-row tile column sums, csum[(m / 128) * csum_ld + n],
 * of the accumulator (PLAIN / ADDSCALE / RELU_MASK, before bias) or of both GATE_BWD outputs
 * (n < 2C, Y's column space) -- the DiffNet backward's per-sequence dilated-conv input-grad
 * sums and gate bias gradients without a pass over Y.  Order: per column, the 8 row groups
 * g (rows g, g+8, ..) summed in row order, then the groups in order; ensvs_tile_colsum computes
 * the same sums, bit for bit, from a Y written by any other path.  Y may be NULL for GATE
 * with ybf and for GATE_BWD with ybf or csum (the fp32 output is not needed). */
int ensvs_tile_colsum(const float* y, int ldy, int M, int N, float* out, int ldo, void* stream);
/* y[m][k] = bf16(x[m][k] + radd[m / T][k]) (radd optional), K % 8 == 0; without radd K may
 * be any size: columns K .. 8*ceil(K/8) - 1 of y are then zero (ldy >= that width). */
int ensvs_cast_bf16(const float* x, int ldx, const float* radd, int radd_ld, int T, long long M,
                    int K, void* y, int ldy, void* stream);

/* Weight gradient of the same contraction (autograd of nn.Conv1d/nn.Linear weights).
 * accum: bit 0 adds into dst (else overwrites); bit 1 (ENSVS_WGRAD_DEFER) with splits > 1 only
 * writes the split partials [splits][taps][N][K] into `part` -- the caller reduces them later,
 * many weight gradients in one launch, with ensvs_wgrad_reduce_batch (same summation order,
 * same bits as the reduction the call would have launched). */
#define ENSVS_WGRAD_DEFER 2
int ensvs_conv_wgrad(const float* dy, int ldy, const float* x, int ldx, const float* radd,
                     int radd_ld, int B, int Tout, int Tin, int N, int K, int taps, int dil,
                     int shift0, int pad, int splits, float* part, float* dst, long long sn,
                     long long sk, long long sj, int accum, float scale, int dtype, void* stream);

/* ensvs_conv_wgrad with bf16 operands (dy, x already rounded to bf16, radd folded into x;
 * ldy, ldx multiples of 8): identical bits, operands staged by global_load_lds.  K (N) need
 * not be a multiple of 8 when every x (dy) row holds K (N) rounded up to 8 readable columns
 * (ldx, ldy >= that): the columns past K (N) are read in the last 16-B chunk and only feed
 * outputs that are never written (the SeparateF0 decoders' 1 026-column input, zero-padded
 * to 1 032; the odd-width fp32 operands' padded copies, kernels.WGRAD_CAST). */
int ensvs_conv_wgrad_bf16(const void* dy, int ldy, const void* x, int ldx, int B, int Tout,
                          int Tin, int N, int K, int taps, int dil, int shift0, int pad, int splits,
                          float* part, float* dst, long long sn, long long sk, long long sj,
                          int accum, float scale, void* stream);

/* Deferred split reductions of ENSVS_WGRAD_DEFER weight gradients, n descriptors (a HOST
 * array, passed by value to the kernels in chunks of 48): dst[n*sn + k*sk + j*sj] (+)= scale *
 * sum over s of part[s][j][n][k], splits summed in order.  The destinations of one call must
 * not overlap (one thread per destination element). */
typedef struct {
  const float* part;
  float* dst;
  long long sn, sk, sj;
  int splits, taps, N, K, accum;
  float scale;
} ensvs_wred_desc;
int ensvs_wgrad_reduce_batch(const ensvs_wred_desc* descs, int n, void* stream);
/* Column sums of several parameter gradients in two launches (the deferred bias gradients
 * of a training step: kernels.deferred_wgrad queues them, flush_wgrad issues them):
 * out[n] (+)= scale * sum over the M rows of y[row * ld + n], with ensvs_colsum's split count
 * for max_splits, rows per split and summation order -- the same bits as one ensvs_colsum
 * (groups 1, no mean) per descriptor.  Descriptors must not share output elements.  `part`:
 * ensvs_colsum_batch_part_floats(descs, n) floats.  Replaces the per-layer
 * `grad_bias = dy.sum(0)` reductions of the reference's autograd (e.g. nn.Linear / nn.Conv1d
 * bias gradients in nnsvs/model.py FFConvLSTM, denoiser.py). */
typedef struct {
  const float* y;
  float* out;
  int ld, M, N, max_splits;
  float scale;
  int accum;
} ensvs_colsum_desc;
long long ensvs_colsum_batch_part_floats(const ensvs_colsum_desc* descs, int n);
int ensvs_colsum_batch(const ensvs_colsum_desc* descs, int n, float* part, long long part_floats,
                       void* stream);

/* Batched weight repack (descs is a DEVICE array). */
int ensvs_pack_weights(const ensvs_pack_desc* descs, int n, int max_elems, void* stream);
/* The same repack as ensvs_pack_weights (the same bits), one workgroup per 64 x 64 tile of one
 * tap: descriptor i owns tiles [descs[i].tile0, descs[i].tile0 + taps * cdiv(Npad, 64) *
 * cdiv(Kp, 64)), tile0 ascending from 0, `tiles` the total.  Tiles are read along the source's
 * unit-stride axis and written along the packed rows through LDS (coalesced both ways). */
int ensvs_pack_weights_tiled(const ensvs_pack_desc* descs, int n, int tiles, void* stream);

/* Grouped column sums (bias grads, BatchNorm statistics). */
int ensvs_colsum(const float* y, int ld, int M, int groups, int N, const float* mean, float scale,
                 float* part, int max_splits, float* out, int ldo, int accum, void* stream);
/* ensvs_colsum in one launch (same splits, same bits): the block that finishes a column
 * block's last split reduces its partials.  counters: cdiv(N, 64) * groups zero-initialised
 * words, left zero by every launch (reuse them on one stream; give concurrent streams their
 * own). */
int ensvs_colsum_once(const float* y, int ld, int M, int groups, int N, const float* mean,
                      float scale, float* part, int max_splits, unsigned* counters, float* out,
                      int ldo, int accum, void* stream);


/* ---- recurrences ------------------------------------------------------ */

/* Packed bidirectional LSTM recurrence, one layer (input projections precomputed
 * by ensvs_conv_gemm into gx [B*T][ldg], dir d gates at cols d*4H + {i,f,g,o}*H).
 * Replaces the time loop of nn.LSTM(bidirectional=True) over pack_padded_sequence:
 * nnsvs/model.py:862-869,914-916 and acoustic_models/tacotron_f0.py:876-883,981-983.
 * Any H >= 1: H in {8,16,32,64,128} runs one persistent workgroup per (sequence,
 * direction); other sizes (the encoders' 256 / 512, the bap decoder's 62 of
 * MultiTrackMultistreamSeparateF0ParametricModel, nnsvs/model.py:1483-1490,861-869) one
 * launch per time step over ceil(H/U) x 2 workgroups.  saved holds [B*T][2][5H]. */
int ensvs_lstm_fwd(const float* gx, int ldg, const float* whh_f, const float* whh_r,
                   const long long* lengths, int B, int T, int H, float* y, int ldy, float* saved,
                   void* stream);
/* Workspace floats ensvs_lstm_bwd needs for (B, H): 2*B*H (cell-gradient carry) for the
 * per-step kernels, 0 for the persistent ones. */
long long ensvs_lstm_bwd_work_floats(int B, int H);
/* Test knob: force != 0 runs the per-step kernels at every H (default 0). */
int ensvs_lstm_set_step(int force);
/* Backward through time: pre-activation gate gradients dg [B*T][lddg] (zero past L_b). */
int ensvs_lstm_bwd(const float* dy, int lddy, const float* whh_f, const float* whh_r,
                   const long long* lengths, int B, int T, int H, const float* saved, float* dg,
                   int lddg, float* work, long long work_floats, void* stream);

/* Cooperative recurrence for H in {256, 512} and B <= 256 in production (bf16 GEMM)
 * precision: one launch for every step, each direction split over H/16 workgroups that keep
 * their W_hh slice in registers and exchange h (fp16) / dG (bf16) through `work` every step
 * (fp16 / bf16 recurrent products, fp32 accumulation, gates, cell state and saved values).
 * Same contract as ensvs_lstm_fwd / ensvs_lstm_bwd (the MultiTrackLSTMEncoder H = 512 and the
 * SeparateF0 decoders' H = 256 of nnsvs/model.py:1483-1490, 861-869).  wpack: W_hh of both
 * directions packed by ensvs_lstm_coop_pack (bwd = 0: forward fp16 fragments, bwd = 1:
 * backward bf16 fragments of W_hh^T), 2*4*H*H 2-byte elements.  Sequences run in tiles of
 * S = ensvs_lstm_coop_tile_seqs(B, H) (blockIdx.z), each tile an independent hand-off group.
 * work: 256-B aligned, ensvs_lstm_coop_work_bytes(H, B) bytes, caller-owned, one per
 * concurrent launch: ceil(B/S) 2 048-B tile headers, then the tiles' slabs; header bytes 128..131 of a tile read non-zero
 * after a launch in which that tile's grid could not become resident (see
 * ensvs_coop_set_error_word for the persistent flag). */
/* MFMA recurrence for H = 64 / 128 in production (bf16 GEMM) precision (lstm_mfma.hip): the
 * structure of the persistent kernels above (one workgroup per (sequence, direction), chunked
 * LDS staging) with the recurrent product h W_hh^T (fp16 fragments) / dG W_hh (bf16) on MFMA,
 * fp32 accumulation, gates, cell state and saved values.  Same contract as ensvs_lstm_fwd /
 * ensvs_lstm_bwd (the FFConvLSTM encoders, nnsvs/model.py:862-869, 914-916; the lf0 encoder,
 * acoustic_models/tacotron_f0.py:876-883).  wpack: ensvs_lstm_mfma_pack output for both
 * directions (bwd = 0: fp16 forward fragments, bwd = 1: bf16 backward fragments of W_hh^T),
 * 2*4*H*H 2-byte elements, 16-B aligned; gx / y / saved / dy / dg 16-B aligned, leading
 * dimensions multiples of 4.  Optional outputs for the bf16-operand GEMMs that consume them
 * (the layer's weight gradients and input gradient), written from the same chunk flush:
 * ybf (bf16 [B*T][ldyb]) = y rounded to bf16; dgbf (bf16 [B*T][lddgb]) = dg rounded to bf16
 * (dg itself may then be NULL, one of the two is required); bsum (fp32 [B][8H]): row b =
 * sum over t of dg row (b, t), the per-sequence partials of the bias gradient (the column
 * sums of dg the reference's autograd forms for b_ih / b_hh).  8-B aligned bf16 pointers. */
int ensvs_lstm_mfma_supported(int H);
int ensvs_lstm_mfma_pack(const float* whh_f, const float* whh_r, int H, int bwd, void* out,
                         void* stream);
int ensvs_lstm_mfma_fwd(const float* gx, int ldg, const void* wpack, const long long* lengths,
                        int B, int T, int H, float* y, int ldy, float* saved, void* ybf,
                        int ldyb, void* stream);
int ensvs_lstm_mfma_bwd(const float* dy, int lddy, const void* wpack, const long long* lengths,
                        int B, int T, int H, const float* saved, float* dg, int lddg,
                        void* dgbf, int lddgb, float* bsum, void* stream);
int ensvs_lstm_coop_supported(int B, int H);
long long ensvs_lstm_coop_work_bytes(int H, int B);
/* Sequences per tile of the cooperative LSTM for a batch of B at hidden size H: 16 while the
 * launch stays within 128 workgroups (H = 512: B <= 32; H = 256: B <= 64) -- every workgroup
 * then reads half the hand-off slab per step -- else 32.  ensvs_lstm_coop_set_tile_seqs(s)
 * forces s in {16, 32} (0: automatic), for A/B runs and tests; set it before sizing `work`. */
int ensvs_lstm_coop_tile_seqs(int B, int H);
int ensvs_lstm_coop_set_tile_seqs(int s);
int ensvs_lstm_coop_pack(const float* whh_f, const float* whh_r, int H, int bwd, void* out,
                         void* stream);
int ensvs_lstm_coop_fwd(const float* gx, int ldg, const void* wpack, const long long* lengths,
                        int B, int T, int H, float* y, int ldy, float* saved, void* work,
                        long long work_bytes, void* stream);
int ensvs_lstm_coop_bwd(const float* dy, int lddy, const void* wpack, const long long* lengths,
                        int B, int T, int H, const float* saved, float* dg, int lddg, void* work,
                        long long work_bytes, void* stream);
/* The same launches with the optional outputs of ensvs_lstm_mfma_fwd / _bwd for the layer's
 * bf16-operand GEMMs (the next layer's input projection, the weight gradients, the input
 * gradient): y16 (bf16 [B*T][ldy16], 8-B aligned, ldy16 % 4 == 0) = y rounded to bf16, written
 * by the forward's service wave with y; dgb (bf16 [B*T][lddgb]) = dg rounded to bf16 -- the
 * bits the backward already hands off -- with dg itself optional (one of the two required);
 * bpart (fp32 [B][8H]) = dg summed over each sequence's steps, the bias gradient's partials.
 * Null optional pointers give the plain entry points above. */
int ensvs_lstm_coop_fwd_ex(const float* gx, int ldg, const void* wpack, const long long* lengths,
                           int B, int T, int H, float* y, int ldy, float* saved, void* y16,
                           int ldy16, void* work, long long work_bytes, void* stream);
int ensvs_lstm_coop_bwd_ex(const float* dy, int lddy, const void* wpack,
                           const long long* lengths, int B, int T, int H, const float* saved,
                           float* dg, int lddg, void* dgb, int lddgb, float* bpart, void* work,
                           long long work_bytes, void* stream);

/* Residual-F0 AR decoder (acoustic_models/tacotron_f0.py:126-237 with
 * ZoneOutCell(LSTMCell), tacotron/decoder.py:20-48).  H in {16,...,256}, T % 4 == 0.
 * teach == NULL: free-running (the multi-track diffusion model, multistream.py:1646-1651,
 * and every inference); teach != NULL: teacher forcing on targets[(b*T + f)*ldt]
 * (BiLSTMResF0NonAttentiveDecoder in training, multistream.py:1158); the backward then
 * takes teacher = 1 (no gradient through the previous output). */
int ensvs_ardec_pack(const float* whh, int H, float* wpf, float* wpb, void* stream);
int ensvs_ardec_fwd(const float* gx, int ldgx, const float* ofx, int ldo, const float* wpf,
                    const float* wih_p, const float* wfo, int ldwfo, const float* score, int lds,
                    const float* mask, const float* teach, int ldt, int B, int T, int H,
                    float in_min, float in_max, float mean, float scale, float* lf0, float* res,
                    float* sg, float* sc, float* sh, float* so, float* sp, void* stream);
int ensvs_ardec_bwd(const float* glf0, const float* gres, const float* wpb, const float* wih_p,
                    const float* wfo, int ldwfo, const float* mask, int teacher, int B, int T,
                    int H, float in_min, float in_max, float mean, float scale, const float* sg,
                    const float* sc, const float* so, float* dg, float* do4, void* stream);
/* Cooperative AR decoder for H in {128, 256}, any B, in production (bf16 GEMM) precision:
 * one launch for all T/4 steps, the recurrence W_hh [h_1 .. h_B] split over H/16 workgroups
 * that keep their W_hh slice in registers (fp16 forward, bf16 W_hh^T backward, fp32
 * accumulation, gates, cell state, feat_out and saved values) and exchange h / dG plus the
 * feat_out / prenet partial sums through `work` every step.  Same contract and saved layout as
 * ensvs_ardec_fwd / ensvs_ardec_bwd (tacotron_f0.py:183-228).  wpack: ensvs_ardec_coop_pack
 * (bwd = 0 forward fp16 fragments, bwd = 1 backward bf16 fragments), 4*H*H 2-byte elements;
 * sequences in tiles of S = ensvs_ardec_coop_tile_seqs(B, H) (blockIdx.y; 16 for B <= 16, else
 * 32; ensvs_ardec_coop_set_tile_seqs forces 16 / 32, 0 automatic) in launches of up to 8 tiles;
 * work: 256-B aligned,
 * ensvs_ardec_coop_work_bytes(H, B) bytes, caller-owned, one per concurrent launch, laid out
 * and flagged as the LSTM's.  The forward's saved-state outputs sg / sc / sh are 16-B aligned
 * (written with 16-B stores). */
int ensvs_ardec_coop_supported(int B, int H);
long long ensvs_ardec_coop_work_bytes(int H, int B);
int ensvs_ardec_coop_tile_seqs(int B, int H);
int ensvs_ardec_coop_set_tile_seqs(int s);
/* Failure controls of every cooperative launch (coop.h).  A tile whose workgroups cannot all
 * become resident times out after `us` microseconds (default 1 s) of polling, releases its
 * waiters (the launch ends within one timeout) and ORs 1 into the registered persistent device
 * word of the launching thread's current device (4-B aligned, caller-owned, never cleared by
 * the library; NULL unregisters).  One word per device: ensvs_coop_set_error_word_dev
 * registers `device`'s word (0..63), ensvs_coop_set_error_word the current device's, and
 * ensvs_coop_error_word returns what is registered for `device` (host-side bookkeeping only, no
 * HIP call).  The word is read by ensvs_l2norm_chk (which also snapshots and clears it once
 * per step), so the training step skips its update.
 * ensvs_coop_inject_fault(1) is a test switch: workgroup 0 of tile 0 skips its step-1 signal. */
int ensvs_coop_set_error_word(unsigned* word);
int ensvs_coop_set_error_word_dev(int device, unsigned* word);
unsigned* ensvs_coop_error_word(int device);
int ensvs_coop_set_timeout_us(long long us);
int ensvs_coop_inject_fault(int on);
int ensvs_ardec_coop_pack(const float* whh, int H, int bwd, void* out, void* stream);
int ensvs_ardec_coop_fwd(const float* gx, int ldgx, const float* ofx, int ldo, const void* wpack,
                         const float* wih_p, const float* wfo, int ldwfo, const float* score,
                         int lds, const float* mask, const float* teach, int ldt, int B, int T,
                         int H, float in_min, float in_max, float mean, float scale, float* lf0,
                         float* res, float* sg, float* sc, float* sh, float* so, float* sp,
                         void* work, long long work_bytes, void* stream);
int ensvs_ardec_coop_bwd(const float* glf0, const float* gres, const void* wpack,
                         const float* wih_p, const float* wfo, int ldwfo, const float* mask,
                         int teacher, int B, int T, int H, float in_min, float in_max, float mean,
                         float scale, const float* sg, const float* sc, const float* so, float* dg,
                         float* do4, void* work, long long work_bytes, void* stream);
/* Depthwise Conv1d(k=4, s=4, groups=C) down-sampling (tacotron_f0.py:104-111,161-164). */
int ensvs_downsample_fwd(const float* p0, int ld0, int n0, const float* p1, int ld1, int n1,
                         const float* p2, int ld2, int n2, const float* w, const float* bias, int B,
                         int T, float* e, int lde, void* stream);
int ensvs_downsample_bwd(const float* de, int lde, const float* p0, int ld0, int n0,
                         const float* p1, int ld1, int n1, const float* p2, int ld2, int n2,
                         const float* w, int B, int T, float* dx, int lddx, float* dw, float* db,
                         void* stream);

/* ---- memory-bound kernels --------------------------------------------- */

/* torch.argmax over the phoneme one-hot columns (model.py:905, tacotron_f0.py:939). */
int ensvs_phoneme_ids(const float* x, int ld, long long M, int ph0, int nv, int* ids,
                      void* stream);
/* y += emb[ids0] (+ emb[ids1]) + spk0[b] (+ spk1[b])  (nn.Embedding + speaker add,
 * model.py:906-910, tacotron_f0.py:941-965). */
int ensvs_embed_add(float* y, int ldy, long long M, int C, int T, const float* emb,
                    const int* ids0, const int* ids1, const float* spk0, const float* spk1,
                    int ldspk, void* stream);
/* demb[ids[m]] += dy[m] over frames (nn.Embedding backward), deterministic: frame
 * chunks accumulate in LDS, partials (>= ensvs_embed_bwd_workspace floats) are summed
 * in a fixed order.  V = vocabulary rows (<= 128). */
int ensvs_embed_bwd(const float* dy, int ldy, long long M, int C, const int* ids, int V,
                    float* part, float* demb, void* stream);
long long ensvs_embed_bwd_workspace(long long M, int C, int V);
/* SpeakerEmbedding (model.py:35-53): gather / scatter-add of table rows. */
int ensvs_spk_scatter(const float* dseq, int B, int C, const long long* spk, float* dtab,
                      void* stream);
int ensvs_gather_rows(const float* table, const long long* idx, int B, int C, float* out,
                      void* stream);
/* BatchNorm1d training mode (model.py:846-859): finalize stats + running update,
 * apply+ReLU, and backward (+ReLU).  Groups of Mg rows keep separate statistics. */
int ensvs_bn_finalize(float* mean, float* var, int G, int C, long long Mg, float eps, float* rstd,
                      float* rmean, float* rvar, float momentum, int update, void* stream);

/* BatchNorm1d training statistics of y [M][ldy] in groups of Mg rows in two launches (the two
 * column sums + ensvs_bn_finalize they replace): mean / var (biased) [G][C], rstd = 1 /
 * sqrt(var + eps), and with updates > 0 the running statistics updated `updates` times per
 * group (bn_finalize's order) and *nbt (the module's num_batches_tracked, int64) += G * updates.
 * part: ensvs_bn_stats_part_floats(M, C, Mg) floats of workspace.  Per row split the column
 * sums and the squared deviations from the split's own mean; merged in a fixed order (Chan's
 * parallel variance, double): deterministic (nnsvs/model.py:837-859 nn.BatchNorm1d). */
long long ensvs_bn_stats_part_floats(long long M, int C, long long Mg);
int ensvs_bn_stats(const float* y, int ldy, long long M, int C, long long Mg, float* part,
                   long long part_floats, float eps, float* mean, float* var, float* rstd,
                   float* rmean, float* rvar, float momentum, int updates, long long* nbt,
                   void* stream);
/* outb / dyb (optional, bf16, 8-B aligned rows, ld % 4 == 0; C % 4 == 0 and 16-B aligned fp32
 * operands, else ENSVS_E_ARG): the output / input gradient also rounded to bf16 for the
 * next convolution's bf16-operand GEMMs (forward input, dgrad, weight gradient). */
int ensvs_bn_apply_relu(const float* y, int ldy, long long M, int C, long long Mg,
                        const float* mean, const float* rstd, const float* gamma,
                        const float* beta, float* out, int ldo, void* outb, int ldob,
                        void* stream);
int ensvs_bn_bwd(const float* dout, int ldd, const float* y, int ldy, long long M, int C,
                 long long Mg, const float* mean, const float* rstd, const float* gamma,
                 const float* beta, float* part, int max_splits, float* sums, float* dgamma,
                 float* dbeta, float* dy, int lddy, void* dyb, int lddyb, void* stream);
/* BatchNorm1d in eval mode inside a training step (model.train() + bn.eval(): frozen running
 * statistics; the data-parallel parity definition, SURVEY 8(e), train_util.py:1176-1182):
 * dgamma/dbeta accumulate, dy = gamma * rstd * dout * (z > 0). */
int ensvs_bn_bwd_frozen(const float* dout, int ldd, const float* y, int ldy, long long M, int C,
                        const float* mean, const float* rstd, const float* gamma,
                        const float* beta, float* part, int max_splits, float* sums,
                        float* dgamma, float* dbeta, float* dy, int lddy, void* stream);
/* DiffNet step embedding (denoiser.py:9-26). */
int ensvs_sinusoidal(const long long* t, int B, int C, float* out, void* stream);
int ensvs_mish_fwd(const float* x, float* y, long long n, void* stream);
int ensvs_mish_bwd(const float* x, const float* dy, float* dx, long long n, void* stream);
/* GaussianDiffusion q_sample (diffusion.py:261-267,289-295) and one p_sample step
 * (diffusion.py:170-204). */
int ensvs_q_sample(const float* y, int ldy, const float* noise, int ldn, const long long* t,
                   const float* sa, const float* s1ma, long long M, int Mc, int T, float inv_ns,
                   float* xn, int ldx, void* stream);
int ensvs_p_sample(float* x, const float* eps, const float* noise, long long n, float sra,
                   float srm1, float c1, float c2, float sigma, void* stream);
/* p_sample over x [M][Mc] that also writes the next denoiser input's bf16 GEMM operand
 * xb [M][ldb] (ldb % 8 == 0, >= Mc; columns Mc..ldb-1 zero: the operand's K padding).
 * eps == NULL: x unchanged, only the copy (the draw x_K before the first step). */
int ensvs_p_sample_bf16(float* x, const float* eps, const float* noise, long long M, int Mc,
                        float sra, float srm1, float c1, float c2, float sigma, void* xb,
                        int ldb, void* stream);
/* Masked L1 loss summed over streams / N with its gradient fused
 * (bin/train_acoustic_multitrack.py:115-173).  loss = invN * sum|a-b| over valid
 * frames; ga = gscale * invN * sign(a-b) (0 on padding).  gscale = 1/world folds the
 * data-parallel gradient average into the loss gradient, so the RCCL all-reduce is a
 * plain sum. */
int ensvs_masked_l1(const float* const* a, const float* const* b, float* const* ga,
                    const int* lda, const int* ldb, const int* ldg, const int* n, int ns,
                    const long long* lengths, int B, int T, float invN, float gscale,
                    float* part, float* loss_out, void* stream);
/* Log-F0 interaction loss between the main and sub tracks of a pair
 * (bin/train_acoustic_multitrack.py:175-182; output_subtrack model, logf0_diff_weight > 0):
 * loss_out += weight * mean over {t < len_b, vuv_main > 0, vuv_sub > 0} of
 * |(lf0_m - lf0_s) - (y_m[lf0_col] - y_s[lf0_col])|; g_m += gscale*weight*sign/N (accumulated
 * onto the masked-L1 gradient), g_s = -(same).  y_m / y_s: target rows (ldy); part >= 1024
 * floats.  lf0_m / lf0_s / g_m / g_s: (B*T) contiguous. */
int ensvs_lf0_interaction(const float* lf0_m, const float* lf0_s, const float* y_m,
                          const float* y_s, int ldy, int lf0_col, int vuv_col,
                          const long long* lengths, int B, int T, float weight, float gscale,
                          float* part, float* loss_out, float* g_m, float* g_s, void* stream);
/* clip_grad_norm_ + torch.optim.Adam over the flat parameter buffer
 * (bin/train_acoustic_multitrack.py:369-380). */
int ensvs_l2norm(const float* x, long long n, float* part, float* norm_out, void* stream);
/* ensvs_l2norm whose result is NaN when err[0] != 0 (a failed cooperative recurrence, see
 * ensvs_coop_set_error_word): the non-finite-norm skip then drops the step's update.  err
 * points at two words: a set err[0] is cleared and counted into err[1] (the host reads and
 * clears err[1] when it raises), so only the step whose recurrence failed skips. */
int ensvs_l2norm_chk(const float* x, long long n, float* part, float* norm_out,
                     unsigned* err, void* stream);
/* x[0] = NaN when *err != 0: before a data-parallel all-reduce, so every rank's norm is NaN
 * and every rank skips the update when any rank's recurrence failed. */
int ensvs_poison_on_error(const unsigned* err, float* x, void* stream);
int ensvs_adam(float* p, float* g, float* m, float* v, long long n, const float* norm,
               float max_norm, float lr, float b1, float b2, float eps, float bc1,
               float sqrt_bc2, void* stream);
/* Graph-replayable clip + Adam: state = {step, lr / (1 - b1^step), sqrt(1 - b2^step), lr}
   (4 doubles on the device; the host sets state[3] = lr).  The step advances on the
   device only when *norm is finite (train_acoustic_multitrack.py:365-380 skips
   optimizer.step()); replaces the torch.optim.Adam step of train_acoustic_multitrack.py:382. */
int ensvs_adam_step(float* p, float* g, float* m, float* v, long long n, const float* norm,
                    float max_norm, double b1, double b2, float eps, double* state, void* stream);
/* Advance the RNG replay epoch (randn / randint / dropout masks): a captured step calls it
   first so every replay draws fresh numbers; epoch 0 (eager) leaves seeds unchanged. */
int ensvs_rng_advance(void* stream);
int ensvs_copy_cols(const float* src, int lds, float* dst, int ldd, long long M, int n,
                    void* stream);
/* dst[m*ldd + b*dw + c] = c < sw ? src[m*lds + b*sw + c] : 0, b < nblk, c < dw: per-gate
 * column blocks widened with zero padding (sw < dw) or narrowed (sw > dw).  The LSTM layers
 * of hidden size 62 (the SeparateF0 bap decoder, nnsvs/model.py:861-869) run the exact fp32
 * persistent H = 64 kernels on zero-padded gates (padded units keep c = h = 0). */
int ensvs_regroup_cols(const float* src, int lds, float* dst, int ldd, long long M, int nblk,
                       int sw, int dw, void* stream);
int ensvs_axpy(float* y, const float* x, float a, long long n, void* stream);
/* y[g*ystride + j] += a * x[g*xstride + j] for g < count, j < n (same-shaped parameters of
 * several layers, e.g. the 20 DiffNet residual blocks' bias gradients, in one launch). */
int ensvs_axpy_strided(float* y, long long ystride, const float* x, long long xstride, float a,
                       int n, int count, void* stream);
/* y[g*ystride + r*yld + c] += a * x[g*xstride + r*xld + c] for g < count, r < rows, c < cols
 * (per-block views of one all-blocks weight gradient, e.g. the skip half of the 20 DiffNet
 * output projections taken as dss^T [z_0 .. z_19]; diffsinger.py:70-110 ResidualBlock). */
int ensvs_axpy_blocks2d(float* y, long long ystride, long long yld, const float* x,
                        long long xstride, long long xld, float a, int rows, int cols, int count,
                        void* stream);
/* DiffNet residual-half output-projection bias grads: with s_l = a*s_{l+1} + cdy[l*C + c]
 * (s = column sums of d x_l, cdy[l] = column sums of the dilated-conv input grad of block l),
 * dst[(l-1)*dstride + c] += a*s_l for l = L-1 .. 1.  Replaces the per-block bias reduction of
 * autograd over diffsinger.py ResidualBlock.forward's output_projection. */
int ensvs_res_bias_grad(const float* cdy, int L, int C, float* dst, long long dstride, float a,
                        void* stream);
/* y = a*y + b*x ; y *= x (dropout masks) */
int ensvs_axpby(float* y, float a, const float* x, float b, long long n, void* stream);
/* out = a*y + b*x, bitwise the same as ensvs_axpby but out of place. */
int ensvs_axpby_to(float* out, const float* y, float a, const float* x, float b, long long n,
                   void* stream);
/* ensvs_axpby_to plus outb[i] = bf16(out[i]) (the next GEMM's pre-rounded operand). */
int ensvs_axpby_to_bf16(float* out, void* outb, const float* y, float a, const float* x, float b,
                        long long n, void* stream);
int ensvs_mul(float* y, const float* x, long long n, void* stream);
int ensvs_mul_out(float* out, const float* a, const float* b, long long n, void* stream);
/* out = act > 0 ? dy : 0 (ReLU backward; out may alias dy); outb (optional, bf16): its copy
 * for the bf16-operand GEMMs (n % 4 == 0, 16-B aligned fp32 pointers, 8-B aligned outb) */
int ensvs_relu_mask(float* out, void* outb, const float* dy, const float* act, long long n,
                    void* stream);
/* Gradient of ReflectionPad1d(pad) (model.py:846-859): dx[b][t] from dxp[b][T+2pad]. */
int ensvs_reflect_fold(const float* dxp, int B, int T, int pad, int C, float* dx, void* stream);
/* Counter-based RNG (stateless hash of (seed, index)): N(0,1), keep-masks scaled by
 * 1/(1-p) (F.dropout), and uniform integers in [0, hi) (torch.randint). */
int ensvs_randn(float* out, long long n, unsigned long long seed, void* stream);
int ensvs_dropout_mask(float* out, long long n, float p, unsigned long long seed, void* stream);
int ensvs_randint(long long* out, long long n, long long hi, unsigned long long seed,
                  void* stream);

/* ---- uSFGAN vocoder (synthesis) ----------------------------------------- */

/* nn.utils.weight_norm folding (usfgan/models/generator.py:524-544, util.py:414):
 * w[n*sn + k*sk] = v[n][k] * (g[n] / ||v[n][:]||) over rows of K contiguous elements;
 * g == NULL copies v (plain weights into the same strided destination). */
int ensvs_weight_norm(const float* g, const float* v, int N, int K, float* w, long long sn,
                      long long sk, void* stream);
/* One stage of UpsampleNetwork (usfgan/layers/upsample.py:86-128): nearest x s along time
 * (F.interpolate scale_factor, inv_s = float(1/s)) then Conv2d(1,1,(1,2s+1), padding (0,s))
 * with taps w.  x (B*Tin, ld) -> y (B*Tin*s, ld); channels C..ld-1 of y are zeroed. */
int ensvs_usf_upsample(const float* x, int ld, int B, int Tin, int C, int s, float inv_s,
                       const float* w, float* y, void* stream);
/* dilated_factor + repeat(hop) (usfgan/utils/features.py:56-75, usfgan/__init__.py:50-58):
 * d[b*T*hop + i] = float((fs / f0') / dense), f0' = f0[b][i/hop] (0 -> fs/dense). */
int ensvs_usf_dfactor(const float* f0, int B, int T, int hop, double fs, double dense, float* d,
                      void* stream);
/* SignalGenerator(["sine", "noise"]) (usfgan/utils/features.py:112-164): out (B*T*hop, ldo)
 * columns [sine + amp*sine_noise, noise]; scale = float(T)/float(T*hop) (nearest upsample of
 * f0); the phase cumsum is scanned in fp64.  ws: ensvs_usf_source_workspace() doubles. */
long long ensvs_usf_source_workspace(int B, int T, int hop);
int ensvs_usf_source(const float* f0, int B, int T, int hop, float scale, float fs,
                     float sine_amp, float noise_amp, const float* sine_noise, const float* noise,
                     double* ws, float* out, int ldo, void* stream);
/* Harmonic/noise mix (usfgan/models/generator.py:505-508): s = a*h + (1-a)*n; keep != 0 also
 * stores h = a*h and n = (1-a)*n (the forward's debug outputs). */
int ensvs_usf_mix(const float* a, float* h, float* n, float* s, long long total, int keep,
                  void* stream);

/* ---- timing models (duration / time-lag) -------------------------------- */

/* MDN head (nnsvs/mdn.py).  Per item = frame (or frame x output dim when dim_wise), the G
 * mixture components live in one lane group of the wavefront (xor-shuffle reductions).
 * Layouts: log_pi [M][G] (dim_wise: [M][G][D]), log_sigma / mu [M][G][D], target [M][ldt].
 * G <= 64. */
/* log_softmax over the mixture, in place (MDNLayer.forward, mdn.py:62-70) and its backward
 * (g <- g - exp(y) * sum(g), in place). */
int ensvs_mdn_log_softmax(float* lp, long long M, int G, int D, int dim_wise, void* stream);
int ensvs_mdn_log_softmax_bwd(const float* y, float* g, long long M, int G, int D, int dim_wise,
                              void* stream);
/* mdn_loss(reduce=False) (mdn.py:78-154) -> loss [items]; with gloss != NULL also the
 * gradients of sum(gloss * loss) w.r.t. log_pi, log_sigma, mu (written). */
int ensvs_mdn_loss(const float* lp, const float* ls, const float* mu, const float* tgt, int ldt,
                   long long M, int G, int D, int dim_wise, float lp_min, float ls_min,
                   float* loss, const float* gloss, float* dlp, float* dls, float* dmu,
                   void* stream);
/* mdn_get_most_probable_sigma_and_mu (mdn.py:167-212): sigma, mu_out [M][D]. */
int ensvs_mdn_most_probable(const float* lp, const float* ls, const float* mu, long long M,
                            int G, int D, int dim_wise, float* sigma, float* mu_out,
                            void* stream);
/* Channel LayerNorm of the VariancePredictor conv stack (nnsvs/layers/layer_norm.py:10-35,
 * model.py:1256; eps 1e-12), one wavefront per frame row; saves mean / rstd per row.  The
 * backward writes dx and dy*xhat [M][C] (column sums: the gamma gradient). */
int ensvs_layer_norm_fwd(const float* x, int ldx, long long M, int C, const float* gamma,
                         const float* beta, float eps, float* y, int ldy, float* mean,
                         float* rstd, void* stream);
int ensvs_layer_norm_bwd(const float* dy, int lddy, const float* x, int ldx, long long M, int C,
                         const float* gamma, const float* mean, const float* rstd, float* dx,
                         int lddx, float* dyxhat, void* stream);
/* loss.masked_select(mask).mean() of the timing train step (bin/train_multitrack.py:113-121):
 * out[0] = mean of x[i] over mask[i] != 0, out[1] = the count (part >= 1024 floats).  The
 * backward writes dx[i] = mask[i] ? gout[0] / out[1] : 0. */
int ensvs_masked_mean(const float* x, const unsigned char* mask, long long n, float* part,
                      float* out, void* stream);
int ensvs_masked_mean_bwd(const unsigned char* mask, long long n, const float* gout,
                          const float* fwd_out, float* dx, void* stream);

/* ---- Transformer encoder (model.py:1540-1671, transformer/encoder.py:82-142,
 * transformer/attentions.py:22-214; attention.hip).  Replaces MultiHeadAttention.attention's
 * torch.matmul / softmax / relative-position reshapes (attentions.py:86-135) and their
 * autograd.  Q / K / V are frame rows [(b*T + t)*ld + h*dk + d]; scores [(b*H + h)][T][T]. */
/* Batched fp32 GEMM C[z](m,n) (=|+=) alpha sum_k A[z](m,k) B[z](k,n), z = zb*H + zh, every
 * operand addressed base + zb*sb + zh*sh + row*sr + col*sc (the per-head score / context
 * products and their transposes). */
int ensvs_bgemm(const float* a, long long asb, long long ash, long long asr, long long asc,
                const float* b, long long bsb, long long bsh, long long bsr, long long bsc,
                float* c, long long csb, long long csh, long long csr, long long csc, int Bn,
                int H, int M, int N, int K, float alpha, int accum, void* stream);
/* The same product with bf16 operands (rounded while staged) and fp32 accumulation on the
 * MFMA units: the production-precision form (the reference recipe's fp16 autocast runs these
 * torch.matmul calls in half precision).  Each operand needs a unit stride on its row or
 * reduction axis, 16-B aligned base and strides that are multiples of 4 floats; other
 * layouts run ensvs_bgemm. */
int ensvs_bgemm_bf16(const float* a, long long asb, long long ash, long long asr, long long asc,
                     const float* b, long long bsb, long long bsh, long long bsr, long long bsc,
                     float* c, long long csb, long long csh, long long csr, long long csc, int Bn,
                     int H, int M, int N, int K, float alpha, int accum, void* stream);
/* y = x / s (the query scaling query / sqrt(k_channels), attentions.py:93). */
int ensvs_div(const float* x, int ldx, float* y, int ldy, long long M, int C, float s,
              void* stream);
/* S += relative-key logits qs_i . ek[j-i+w] (|j-i| <= w), masked_fill(-1e4) where i or j is
 * past the length, softmax over j in place; keep (dropout keep-mask, scaled) -> Pd = P*keep. */
int ensvs_attn_softmax(float* S, const float* qs, int ldq, const float* ek,
                       const long long* lens, int B, int H, int T, int dk, int w,
                       const float* keep, float* Pd, void* stream);
/* O += sum_{|j-i|<=w} P[i][j] ev[j-i+w] (_matmul_with_relative_values, attentions.py:124-131) */
int ensvs_attn_relv(const float* P, const float* ev, float* O, int ldo, int B, int H, int T,
                    int dk, int w, void* stream);
/* D[row][i+r-w] += vec_i . tab[r] (band of dO ev^T in the backward) */
int ensvs_attn_band_dot(float* D, const float* vec, int ldv, const float* tab, int B, int H,
                        int T, int dk, int w, void* stream);
long long ensvs_attn_table_grad_workspace(int dk, int w);
/* out[r][d] (+)= sum over rows A[row][i+r-w] X_i[d]: emb_rel_v / emb_rel_k gradients */
int ensvs_attn_table_grad(const float* A, const float* X, int ldx, int B, int H, int T, int dk,
                          int w, float* part, float* out, int accum, void* stream);
/* in place dS = P (dPd*keep - sum_j P dPd*keep), 0 at masked scores */
int ensvs_attn_softmax_bwd(float* dS, const float* P, const float* keep, const long long* lens,
                           int B, int H, int T, void* stream);
/* out_i += sum_r A[row][i+r-w] tab[r] (relative-key part of dQ) */
int ensvs_attn_band_rows(const float* A, const float* tab, float* out, int ldo, int B, int H,
                         int T, int dk, int w, void* stream);
/* y = x * x_mask (sequence_mask of lengths over frame rows; y may alias x) */
int ensvs_mask_rows(const float* x, int ldx, float* y, int ldy, int B, int T, int C,
                    const long long* lens, void* stream);
/* x[:, off::r] (bwd = 0) / its scatter-back with zeros (bwd = 1), model.py:1660 */
int ensvs_stride_rows(const float* x, int ldx, float* y, int ldy, int B, int T, int C, int r,
                      int off, int bwd, void* stream);
/* conv_downsample: depthwise Conv1d(C, C, r, stride=r, groups=C) (model.py:1610-1617), and
 * its backward: dx, and prod[b*Tp+tp][c*r+k] = dy*x whose column sums are dw. */
int ensvs_dwdown_fwd(const float* x, int ldx, const float* w, const float* bias, float* y,
                     int ldy, int B, int T, int C, int r, void* stream);
int ensvs_dwdown_bwd(const float* dy, int ldy, const float* x, int ldx, const float* w,
                     float* dx, int lddx, float* prod, int B, int T, int C, int r, void* stream);

/* ---- Post-acoustic feature processing (gen.py postprocess_acoustic :1314-1530; row f4;
 * postprocess.hip).  Frame rows [t*ld + c], in place. */
/* variance_scaling (postfilters.py:9-46) of columns [offset, D) over the frames with
 * note[t] != 0 (get_note_frame_indices, io/hts.py:29-45); gv: float64 [D] (scaler var_). */
int ensvs_gv_scale(float* x, int ld, int T, int D, int offset, const unsigned char* note,
                   const double* gv, void* stream);
/* gen_spsvs_static_features' F0 stream (gen.py:1988-2016, relative_f0 = False): vuv
 * threshold, exp/log round trip, nnmnkwii interp1d(slinear) over unvoiced frames, + shift.
 * work: T floats. */
int ensvs_world_lf0(float* lf0, int ldl, const float* vuv, int ldv, int T, float thr,
                    float shift, float* work, void* stream);
/* lowpass_filter (dsp.py:10-33): scipy.signal.filtfilt(b, a, x) per column, float64; ba =
 * [b | a] (nb each), zi = lfilter_zi(b, a) (nb - 1), padlen = 3 nb; columns are left unchanged
 * when T <= guard.  work: C * (T + 2 padlen) doubles. */
int ensvs_filtfilt(float* x, int ld, int T, int C, const double* ba, int nb, const double* zi,
                   int padlen, int guard, double* work, void* stream);
/* ngroups (<= 4) ensvs_filtfilt calls with nb = 6 on column groups of one matrix, in one
 * launch: group i filters columns cols[i] .. cols[i] + C[i] - 1 with ba[i], zi[i], padlen[i],
 * guard[i] and workspace work[i] (the post-filter's independent lf0 / mgc / bap smoothing). */
int ensvs_filtfilt_multi(float* x, int ld, int T, int ngroups, const int* cols, const int* C,
                         const double* const* ba, const double* const* zi, const int* padlen,
                         const int* guard, double* const* work, void* stream);
/* bap clip [-60, 0] (gen.py:1520-1522) and the WORLD aperiodicity codec round trip before
 * uSFGAN (gen.py:1649-1670). */
int ensvs_bap_post(float* bap, int ld, int T, int D, int clip, int codec, void* stream);
/* note[t] = score[t * lds] > 0: the note frames of the GV post-filter (gen.py:1339-1340). */
int ensvs_note_mask(const float* score, int lds, int T, unsigned char* note, void* stream);
/* f0[t] = exp(lf0[t * ldl]), 0 where vuv[t * ldv] < thr when zero_unvoiced: the uSFGAN sine
 * source F0 (gen.py:1662-1666). */
int ensvs_f0_from_lf0(const float* lf0, int ldl, const float* vuv, int ldv, int T, float thr,
                      int zero_unvoiced, float* f0, void* stream);
/* sklearn scaler arithmetic in place (float32 data, float64 statistics a, b per column):
 * mode 0 x = x*a + b (StandardScaler.inverse_transform, gen.py:1299; MinMaxScaler.transform),
 * mode 1 x = (x - b)/a (StandardScaler.transform: the vocoder input scaler, gen.py:1678-1684). */
int ensvs_scale_cols(float* x, int ld, int T, int C, const double* a, const double* b, int mode,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ENSVS_H_ */
