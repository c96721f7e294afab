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
       ENSVS_EPI_ADDSCALE = 4 };

/* One K-segment of the implicit-GEMM activation operand. */
typedef struct ensvs_conv_seg {
  const float* x;     /* frame rows (offset to the segment's first channel) */
  const float* radd;  /* optional per-sequence vector added to in-range values */
  long long wofs;     /* element offset of packed weights [taps][Npad][Kp] */
  int ld, K, taps, dil, shift0, pad, radd_ld, Tin, Kp;
} ensvs_conv_seg;

/* Weight repack descriptor (reference layout -> GEMM layout [tap][Npad][Kp]). */
typedef struct ensvs_pack_desc {
  const float* src;
  const float* src2;
  void* dst;
  long long sn, sk, sj;
  int N, K, taps, Npad, Kp, perm_c, flip, transpose, dtype;
  float scale;
} ensvs_pack_desc;

/* Conv1d / Linear forward and input-gradient as an MFMA implicit GEMM.
 * Replaces nn.Conv1d / nn.Linear / nn.ReflectionPad1d call sites in
 * nnsvs/model.py:837-859 (FFConvLSTM.ff/.conv), nnsvs/acoustic_models/tacotron_f0.py:852-874,
 * and the DiffNet convolutions nnsvs/diffsinger/denoiser.py:40-66,101-124. */
int ensvs_conv_gemm(const ensvs_conv_seg* segs, int nseg, int B, int Tout, int N, int Npad,
                    const void* W, int wdtype, const float* bias, float* Y, int ldy, int epi,
                    int relu, int accum, float* aux0, int ld0, const float* aux1, int ld1,
                    float alpha, int C, void* stream);

/* Weight gradient of the same contraction (autograd of nn.Conv1d/nn.Linear weights). */
int ensvs_conv_wgrad(const float* dy, int ldy, const float* x, int ldx, const float* radd,
                     int radd_ld, int B, int Tout, int Tin, int N, int K, int taps, int dil,
                     int shift0, int pad, int splits, float* part, float* dst, long long sn,
                     long long sk, long long sj, int accum, int dtype, void* stream);

/* Batched weight repack (descs is a DEVICE array). */
int ensvs_pack_weights(const ensvs_pack_desc* descs, int n, int max_elems, void* stream);

/* Grouped column sums (bias grads, BatchNorm statistics). */
int ensvs_colsum(const float* y, int ld, int M, int groups, int N, const float* mean, float scale,
                 float* part, int max_splits, float* out, int accum, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ENSVS_H_ */
