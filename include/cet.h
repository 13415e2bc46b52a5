/* cet.h — C ABI of the MI355X channel-prediction engine (libcet.so).
 *
 * Drop-in boundary for the reference's model calls.  Plain pointers and
 * sizes only; device pointers are HIP device memory, `stream` is a hipStream_t
 * (NULL = default stream).  Every function returns 0 on success and a negative code
 * on error; cet_last_error() then describes it (thread-local).  A handle is not
 * thread-safe, and its forwards must not overlap on different streams: the engine's device scratch
 * (table ring, NMSE partials and finish counter, encoder-split exchange) is per handle.  Use one
 * handle per host thread / stream.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   cet_create_informer      InformerStack.__init__ / Informer.__init__
 *                            FullPrecision/InformerModel/model.py:142-245 / :11-113,
 *                            models/InformerLSQ/model.py (LSQ variant, num_bits)
 *   cet_create_transformer   build_transformer  models/Transformer/model.py:90-174
 *   cet_load_weight          nn.Module.load_state_dict (reference key names,
 *                            e.g. "encoder.encoders.0.attn_layers.0.attention.query_projection.weight")
 *                            as used at FullPrecision/QuantizationAwareTraining.py:192-202
 *   cet_set_prob_indices     the torch.randint draw inside ProbAttention._prob_QK
 *                            FullPrecision/InformerModel/attn.py:96-98 (parity mode)
 *   cet_seed                 torch.manual_seed + that draw, reproduced natively (mt19937 % L_K)
 *   cet_forward              InformerStack.forward / Transformer.forward
 *                            FullPrecision/InformerModel/model.py:247-271,
 *                            models/Transformer/model.py:76-87
 *   cet_nmse_split           NMSELossSplit / NMSE_Split_cuda  FullPrecision/metrics.py:26-39
 *   cet_prepare_batch        SeqData.__getitem__ (window, channelnorm, noise) + LoadBatch + the
 *                            callers' decoder input: FullPrecision/dataset.py:124-152, :77-88,
 *                            :54-74, :20-44; QuantizationAwareTraining.py:97-114
 *   cet_synth_channels       stand-in channel source for the absent CDL dataset pickles
 *                            (read by SeqData.__init__, FullPrecision/dataset.py:106-115)
 */
#ifndef CET_H
#define CET_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cet_engine cet_engine;

enum {
  CET_OK = 0,
  CET_E_INVALID = -1,     /* bad argument / unsupported configuration */
  CET_E_MISSING = -2,     /* a required weight was never loaded */
  CET_E_HIP = -3,         /* HIP runtime error */
  CET_E_STATE = -4        /* call out of order (e.g. indices not set) */
};

/* Effective InformerStack flags (after the callers' positional shift). */
typedef struct {
  int enc_in, dec_in, c_out;
  int seq_len, label_len, out_len;
  int factor, d_model, n_heads;
  int n_enc;              /* encoders in the stack (len(e_layers)); 1 for Informer */
  int e_layers[4];
  int d_layers, d_ff;
  int attn_prob;          /* 1: attn == "prob", 0: "full" */
  int distil, mix, output_attention;
  int act_relu;           /* 1: ReLU FFN, 0: GELU */
  int stack;              /* 1: InformerStack (EncoderStack windows), 0: Informer */
  int lsq_bits;           /* 0: full precision; else models/InformerLSQ weight grid */
} cet_informer_config;

typedef struct {
  int src_vocab, tgt_vocab, src_seq_len, tgt_seq_len, label_len, d_model, N, h, d_ff;
} cet_transformer_config;

const char* cet_last_error(void);
int cet_version(void);

int cet_create_informer(const cet_informer_config* cfg, cet_engine** out);
int cet_create_transformer(const cet_transformer_config* cfg, cet_engine** out);
void cet_destroy(cet_engine* e);

/* host fp32 data, `numel` elements, reference state_dict key name */
int cet_load_weight(cet_engine* e, const char* name, const float* data, int64_t numel);
/* number of weights the engine still needs (0 when ready) */
int cet_missing_weights(cet_engine* e, char* first_missing, int buflen);

/* ProbSparse sampling.  cet_prob_calls() returns the number of torch.randint draws one
 * forward makes; shapes[i*3..] = {L_K, L_Q, U} for i < max. */
int cet_prob_calls(cet_engine* e, int* shapes, int max);
/* Explicit draws for the NEXT forward only (parity mode); all calls must be set.  They are consumed
 * by that forward and leave a seeded native stream where it was. */
int cet_set_prob_indices(cet_engine* e, int call, const int32_t* host_idx, int L_Q, int U);
int cet_seed(cet_engine* e, uint64_t seed);          /* switch to the native sampler */
/* Draw one forward's worth of indices (all calls, concatenated, row-major) from the native
 * sampler into host memory, advancing it exactly as cet_forward would; returns the count
 * (out == NULL: only the count). */
int64_t cet_native_draw(cet_engine* e, int32_t* out, int64_t n_max);
/* The draws the NEXT native forward will consume (same layout as cet_native_draw) without
 * advancing the stream: lets a caller replay that forward later with explicit indices. */
int64_t cet_peek_draw(cet_engine* e, int32_t* out, int64_t n_max);

/* Forward on device buffers: x_enc [B][seq_len][enc_in], x_dec [B][label_len+out_len][dec_in]
 * → out [B][out_len][c_out].  attns (optional, Informer with output_attention): per
 * sequence block of cet_attns_floats() floats; layer views via cet_attns_layout(). */
int cet_forward(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, float* attns,
                void* stream);
/* The validation step of run_validation (FullPrecision/QuantizationAwareTraining.py:115-122):
 * out = model(x_enc, x_dec) and NMSELossSplit(out, label) (metrics.py:26-39) in one launch — the
 * v4 kernel computes each sequence's per-step (Σ(x − x̂)², Σx̂²) in its projection epilogue and the
 * last workgroup to finish reduces them over the batch in a fixed order (fp64).  label [B][out_len]
 * [c_out] device fp32; nmse_acc [out_len] fp32 (+= the batch's ratio) and/or nmse_sums [2][out_len]
 * fp64 (the raw sums, overwritten) may be NULL, not both.  Other kernels / c_out > 16: the forward
 * then the standalone reduction on the same stream. */
int cet_forward_nmse(cet_engine* e, const float* x_enc, const float* x_dec, int B, float* out, const float* label,
                     float* nmse_acc, double* nmse_sums, void* stream);
int64_t cet_attns_floats(cet_engine* e);
int cet_attns_layout(cet_engine* e, int64_t* offsets, int* lengths, int max);

/* Debug: per-stage activation dumps into a device buffer of B·cet_debug_floats() floats. */
int cet_set_debug(cet_engine* e, float* dbg_dev);
int64_t cet_debug_floats(cet_engine* e);
int cet_debug_layout(cet_engine* e, char* json, int buflen);
/* Diagnostics (DIAG kernel instance): per-phase s_memtime stamps into a device buffer of B·128 uint64. */
int cet_set_stamps(cet_engine* e, uint64_t* stamps_dev);

/* Select the fused-kernel generation of an Informer engine: 4, the only one (one sequence per 512-thread
 * workgroup, two workgroups per CU, every precision policy, the attention maps and the small-batch
 * encoder split).  Generations 1-3 and 5 (two sequences per workgroup: measured slower)
 * are retired: CET_E_INVALID. */
int cet_set_variant(cet_engine* e, int variant);
/* The kernel path the engine's last Informer forward took: CET_PATH_V4,
 * CET_PATH_V4_SPLIT (v4 with the stack's encoders on separate workgroups), CET_PATH_LW (layer-wise
 * operator launches), CET_PATH_LW_FUSED (the layer-wise forward fused into one launch, one workgroup
 * per sequence with its activations in LDS), 0 before any. */
enum { CET_PATH_LW = 3, CET_PATH_V4 = 4, CET_PATH_LW_FUSED = 31, CET_PATH_V4_SPLIT = 41 };
int cet_last_path(cet_engine* e);
/* The kernel instance the engine's last forward launched, as rocprofv3's kernel trace names it (e.g.
 * "cet::v4::informer_forward_v4<64, false, 0, false, 1, false, false, 0>" for the C2 instance: d_ff, diagnostic
 * outputs, precision, encoder split, the plan's compile-time rows SH (0 generic, 1 C2, 2 the TimingAnalysis
 * e_layers [4, 3] stack), phase stamps, the decoder on the LDS-DMA weight feed, the decoder's precision),
 * written NUL-terminated into
 * name[buflen]; returns its length (0 before any forward, or after a layer-wise forward of several
 * operator launches).  No reference counterpart: measurement plumbing (bench.py's roofline.kernel). */
int cet_last_kernel(cet_engine* e, char* name, int buflen);

/* Operand precision of the v4 kernel's dense layers (Informer engines):
 *   -1 auto (default): 0, or 1 where bf16 cannot carry the model — an LSQ integer grid with |q| > 256,
 *      or a genuinely sparse masked decoder (u < label_len + out_len), whose output is discontinuous
 *      in the top-u selection;
 *    0 bf16 operands, fp32 accumulation / LayerNorm / softmax (the C2 contract);
 *    1 split bf16 (hi + lo per operand, three MFMAs per product): fp32-level parity;
 *    2 fp8 (OCP e4m3) activations on the fp8 MFMA for the LSQ-quantised layers, the integer weight
 *      grid carried exactly as two e4m3 parts (LSQ engines of at most 8 bits);
 *    3 (reported only) the layer-wise engine: models the fused kernels cannot carry (d_model != 128,
 *      n_heads != 8, d_ff > 128, more than 96 encoder / 48 decoder rows; up to d_model 1024 and 128
 *      rows) run as one launch per operator with fp32 operands on the f32 MFMA (cet_lw.hip).
 *      CET_LAYERWISE=1 in the environment at cet_create_informer routes any model there.  On such an
 *      engine "auto" keeps fp32 and 0 selects bf16 GEMM operands (fp32 accumulation, LayerNorm and
 *      attention) in its fused one-launch form (cet_lwf.hip; feature counts multiples of 8): a forward
 *      outside that form then fails with CET_E_INVALID; 1 and 2 are refused.
 *    4 mixed: the encoder in bf16 (two workgroups per CU) and the decoder in split bf16 — for genuinely
 *      sparse masked decoders, whose top-u selection needs fp32-level Q·K (d_ff 64, <= 48 decoder rows).
 * cet_get_precision() returns the precision the packed plan uses (packs the weights if needed).
 * Replaces nothing in the reference, which computes in fp32 (FullPrecision/InformerModel) or with
 * fp32 fake-quantised weights (models/InformerLSQ/LSQ.py:65-74). */
int cet_set_precision(cet_engine* e, int prec);
int cet_get_precision(cet_engine* e);

/* Where the native sampler (after cet_seed) runs: 0 = on the device (the
 * resident mt19937, default), 1 = on the host (the same torch-compatible stream drawn by the host
 * mirror, the multiplicity tables staged per forward through a pinned ring and copied on the
 * caller's stream ahead of the kernel).  Both give identical draws; switching keeps the stream.
 * Replaces nothing in the reference: there the draw is torch.randint on the CPU
 * (FullPrecision/InformerModel/attn.py:96-98), which is what on_host = 1 mirrors. */
int cet_set_sampler(cet_engine* e, int on_host);

/* Kernel timing: when enabled (enable = N ≥ 1), one cet_forward in every N brackets its kernel launch
 * with a pair of hipEvents on the caller's stream; cet_timing_read() waits for them and returns the
 * summed kernel time and the number of bracketed launches since cet_timing(e, N). */
int cet_timing(cet_engine* e, int enable);
int cet_timing_read(cet_engine* e, double* total_ms, int64_t* launches);

/* NMSE_Split_cuda(x_hat=pred, x=label) per prediction step over [B][T][F] fp32 device
 * tensors → out_dev[T] (fp32); if accumulate, out_dev[T] += ratio instead of =. */
int cet_nmse_split(const float* pred, const float* label, int B, int T, int F, float* out_dev, int accumulate,
                   void* stream);
/* The same reduction with its raw fp64 sums: sums_dev[t] = Σ_{b,f}(x − x̂)², sums_dev[T + t] = Σ_{b,f} x̂²
 * (overwritten), so ranks that hold shards of one batch can add their sums before dividing.  out_dev
 * (may be NULL) receives / accumulates the ratio as cet_nmse_split does. */
int cet_nmse_split_sums(const float* pred, const float* label, int B, int T, int F, float* out_dev, int accumulate,
                        double* sums_dev, void* stream);

/* Device channel pipeline.  For b < B, sample s = sample_idx ? sample_idx[b] : sample_base + b of
 * the complex64 dataset [n_samples][slots][nr][nt] (interleaved re, im): normalise to unit mean
 * power over the whole sample, add complex AWGN of variance 10^(-snr_db/10)·(mean power), window
 * slots [st, st + seq_len + pred_len) and write, in LoadBatch layout (feature 2·(r·nt + t) + {re, im}):
 *   x_enc[B][seq_len][2·nr·nt]  the noisy first seq_len slots,
 *   label[B][pred_len][...]     the clean last pred_len slots (may be NULL),
 *   x_dec[B][label_len + pred_len][...]  last label_len encoder slots, then zeros (may be NULL).
 * st = start ? start[b] : a device Philox draw in [0, slots - seq_len - pred_len]; the standard
 * normals are noise[b][slots][nr][nt][2] when given (parity mode: the reference's two torch.randn
 * draws) or Philox4x32-10 / Box-Muller draws keyed by (seed, counter, b, element) otherwise.
 * start_out[B] (may be NULL) receives the windows used.  All arrays are device memory.  A sample
 * index or window outside the dataset yields NaN rows for that sample. */
int cet_prepare_batch(const float* dataset, int64_t n_samples, int slots, int nr, int nt, const int32_t* sample_idx,
                      int64_t sample_base, const int32_t* start, const float* noise, uint64_t seed, uint64_t counter,
                      int B, int seq_len, int label_len, int pred_len, double snr_db, float* x_enc, float* x_dec,
                      float* label, int32_t* start_out, void* stream);

/* Seeded sum-of-sinusoids (Jakes) channels, unit mean power per sample:
 * out[s][t][e] = Σ_p gain[s][e][p]·exp(j(2π·doppler·cos(alpha[s][e][p])·t + phi[s][e][p])) / sqrt(paths),
 * e = r·nt + a; alpha/phi fp32 [n][nr·nt][paths], gain complex64 [n][nr·nt][paths] (re, im),
 * out complex64 [n][slots][nr·nt].  Device memory. */
int cet_synth_channels(const float* alpha, const float* phi, const float* gain, int n, int slots, int nr, int nt,
                       int paths, double doppler, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
