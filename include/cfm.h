/*
 * cfm.h — C-ABI of the MI355X-native ChunkFormer encoder hot path (libcfm.so).
 *
 * Drop-in boundary for the reference's `ChunkFormerEncoder` method set
 * (ishine/chunkformer, chunkformer/modules/encoder.py).  The reference has no
 * FFI of its own: it is plain Python method calls on nn.Modules, so each entry
 * point below names the reference method it replaces; the Python mirror
 * (chunkformer_amd/encoder.py) binds them with ctypes exactly as the
 * reference's callers call the module.
 *
 * Conventions
 *   - every pointer named *_dev / buffer argument is DEVICE memory owned by the
 *     caller (torch tensors in the Python mirror); host arrays are named *_host
 *     or documented as host;
 *   - all device work is stream-ordered on `stream` (a hipStream_t);
 *   - cfm_encode_* and cfm_ctc_* perform no allocation and no host
 *     synchronisation, so they can be captured into a HIP graph;
 *   - one model handle per device, one host thread per device (one
 *     torch.distributed rank per GPU);
 *   - status codes map to the reference's exception types:
 *       CFM_ERR_VALUE   -> ValueError      (bad argument / size)
 *       CFM_ERR_ASSERT  -> AssertionError  (unsupported configuration, encoder.py:94-96,116)
 *       CFM_ERR_RUNTIME -> RuntimeError    (HIP failure, shape mismatch)
 *     cfm_last_error() returns the thread-local message of the last failure.
 */
#ifndef CFM_H
#define CFM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { CFM_OK = 0, CFM_ERR_VALUE = 1, CFM_ERR_ASSERT = 2, CFM_ERR_RUNTIME = 3 } cfm_status;
/* F16: the reference decoder's --autocast_dtype fp16 (chunkformer_model.py:709-743) */
typedef enum { CFM_DTYPE_F32 = 0, CFM_DTYPE_BF16 = 1, CFM_DTYPE_F16 = 2 } cfm_dtype;

/* encoder_conf subset (encoder.py:36-70) + CTC output_dim (init_model.py:73) */
typedef struct {
  int32_t input_dim;      /* 80 */
  int32_t d_model;        /* output_size: 128, 256 or 512 */
  int32_t n_heads;        /* attention_heads: head dim d_model / n_heads must be 64 or 128 */
  int32_t ffn_dim;        /* linear_units */
  int32_t num_blocks;
  int32_t kernel_size;    /* cnn_module_kernel (15) */
  int32_t vocab;          /* CTC output_dim, 0 = no CTC head */
  float norm_eps;         /* 1e-5 */
  int32_t has_cmvn;       /* global_cmvn present */
  int32_t compute_dtype;  /* cfm_dtype: F32 = exact-f32 MFMA parity mode, BF16 / F16 = 16-bit MFMA, f32 accumulate */
} cfm_config;

/* one state_dict tensor, by reference key name, host f32 contiguous */
typedef struct {
  const char* name;
  const float* data;
  int64_t numel;
} cfm_tensor_view;

typedef struct cfm_model cfm_model;
typedef void* cfm_stream; /* hipStream_t */

const char* cfm_version(void);
const char* cfm_last_error(void);

/* Build a model on `device` from reference state_dict tensors (replaces
 * init_speech_model + load_checkpoint for the encoder, init_model.py:61-145,
 * checkpoint.py:26-41).  Weights are repacked into device layouts owned by the
 * handle.  Missing / mis-shaped keys -> CFM_ERR_VALUE. */
cfm_status cfm_model_create(const cfm_config* cfg, const cfm_tensor_view* weights, int32_t n_weights,
                            int32_t device, cfm_model** out);
void cfm_model_destroy(cfm_model* m);
/* diagnostic knobs:
 *   "max_layers"    run only the first N blocks (-1 = all)
 *   "profile"       bitmask of kernel classes to bracket with HIP events on the launch
 *                   stream (bit i = class i of cfm_profile_read); 0 = off
 *   "profile_reset" clear the accumulated profile
 *   "ring_attention" 1 (default) = bf16 masked batch uses the sliding-ring attention kernel,
 *                   0 = the generic per-block kernel (A/B testing)
 *   "fe_fuse_dw2"   1 (default) = bf16 front-end pw1 + ReLU + dw2 in one weight-stationary GEMM,
 *                   0 = pw1 GEMM + the separate dw2 kernel (bit-identical; A/B testing)
 *   "fe_conv"       bf16 conv0 + ReLU + dw1: 6 (default) = channel-stationary, dw1 on MFMA with
 *                   conv0's ReLU output rounded to bf16 (as autocast does), about 5 chunks of 256
 *                   positions per workgroup, balanced per window (2 + k: about k + 1 chunks);
 *                   1 = position-stationary, dw1 in f32 on the VALU
 * (all per-model kernel options: struct Tuning in chunkformer_amd/csrc/cfm_kernels.h, keyed in
 *  cfm_model_set_option, chunkformer_amd/csrc/model.hip) */
cfm_status cfm_model_set_option(cfm_model* m, const char* key, int64_t value);
/* Per kernel class: name, accumulated milliseconds and launch count of the
 * event-bracketed launches since the last reset.  Host-synchronising (waits for
 * the recorded events); never call it inside graph capture.  Returns the number
 * of classes (fills at most `cap`). */
int32_t cfm_profile_read(const cfm_model* m, const char** names, double* total_ms, int64_t* launches, int32_t cap);

/* ------------------------------------------------------------------ plans
 * A plan is an int32 blob computed on the HOST (no GPU needed) and uploaded by
 * the caller; it carries the packer's integer work (chunk windows, masks as
 * [lo, hi) ranges, kernel block descriptors, per-row validity).
 *
 * cfm_plan_masked: the masked-batch packer of forward_parallel_chunk
 * (encoder.py:534-604 + masks 625-645), bit-exact.  Per utterance: lens[b]
 * fbank frames, offsets[b] carried offset (encoder.py:565-594).  Outputs
 * n_chunks[b], out_lens[b] = calc_length(lens[b]) (subsampling.py:270-288),
 * *total_chunks.  Call with plan == NULL to get *plan_ints, then again with a
 * buffer of that many int32. */
cfm_status cfm_plan_masked(const int32_t* lens_host, const int32_t* offsets_host, int32_t B, int32_t chunk_size,
                           int32_t left_context, int32_t right_context, int32_t* n_chunks_host,
                           int32_t* out_lens_host, int32_t* total_chunks, int32_t* plan_host, int64_t* plan_ints);
/* cfm_plan_masked_ex: the same with the feature row count of each utterance (lens_host: x.size(0),
 * which the reference pads and unfolds, encoder.py:556-564) separate from xs_origin_lens
 * (mask_lens_host, NULL = lens_host), which bounds the masks and gives out_lens (encoder.py:567-596,
 * 673).  A length pair whose bound count differs from the window count is the reference's shape
 * mismatch: CFM_ERR_RUNTIME. */
cfm_status cfm_plan_masked_ex(const int32_t* lens_host, const int32_t* mask_lens_host, const int32_t* offsets_host,
                              int32_t B, int32_t chunk_size, int32_t left_context, int32_t right_context,
                              int32_t* n_chunks_host, int32_t* out_lens_host, int32_t* total_chunks, int32_t* plan_host,
                              int64_t* plan_ints);

/* cfm_plan_padded: padded-batch geometry of forward_encoder (encoder.py:220-274,
 * attention.py:334-386, convolution.py:148-167).  chunk_size <= 0 -> full
 * attention.  *t_out = calc_length(T). */
cfm_status cfm_plan_padded(const int32_t* lens_host, int32_t B, int32_t T, int32_t chunk_size, int32_t left_context,
                           int32_t right_context, int32_t* t_out, int32_t* plan_host, int64_t* plan_ints);

/* ------------------------------------------------------------------ encoder
 * cfm_encode_masked replaces ChunkFormerEncoder.forward_parallel_chunk
 * (encoder.py:503-681).  feats_dev: the B utterances' fbank concatenated
 * [sum T_b, 80] f32.  att_cache_in / cnn_cache_in: [nb, L, H, 2*dk] / [nb, d, 7]
 * f32 or NULL (no cache: zeros, and no new cache is produced).  With caches,
 * the new caches (attention.py:466-467, convolution.py:228-230) are written to
 * att_cache_out / cnn_cache_out (may alias the inputs).  out_dev: [N*C, d] f32
 * after after_norm.  workspace: cfm_workspace_bytes_masked() bytes.  plan_host is the
 * host copy of the plan (only its header is read: launch geometry), plan_dev the
 * same blob in device memory (read by the kernels). */
size_t cfm_workspace_bytes_masked(const cfm_model* m, int32_t total_chunks, int32_t chunk_size, int32_t left_context,
                                  int32_t right_context);
cfm_status cfm_encode_masked(const cfm_model* m, const float* feats_dev, const int32_t* plan_host,
                             const int32_t* plan_dev, const float* att_cache_in, const float* cnn_cache_in, int32_t truncated_context_size,
                             float* att_cache_out, float* cnn_cache_out, float* out_dev, void* workspace,
                             size_t workspace_bytes, cfm_stream stream);

/* cfm_encode_masked reading each utterance's fbank where the caller holds it: utt_feats_dev is a
 * DEVICE array of B pointers, utterance b's [x.size(0), 80] f32 rows (the reference's list `xs`,
 * encoder.py:553-564), in the order of the plan's lengths.  Same result as cfm_encode_masked on the
 * concatenation, without the concatenation copy (torch.cat at encoder.py:606). */
cfm_status cfm_encode_masked_utts(const cfm_model* m, const float* const* utt_feats_dev, const int32_t* plan_host,
                                  const int32_t* plan_dev, const float* att_cache_in, const float* cnn_cache_in,
                                  int32_t truncated_context_size, float* att_cache_out, float* cnn_cache_out,
                                  float* out_dev, void* workspace, size_t workspace_bytes, cfm_stream stream);

/* cfm_encode_masked in stages, for pipelining consecutive endless_decode segments (segment k + 1's
 * layer l needs only segment k's layer-l caches): stage -1 = the front-end, relative positions and the
 * first LayerNorm; stage l = encoder layer l (the last one ends with after_norm into out_dev).  Calls
 * over consecutive stage ranges [stage_lo, stage_hi] with the same plan, caches and workspace equal one
 * cfm_encode_masked call bit for bit; the workspace carries the state between them. */
cfm_status cfm_encode_masked_stages(const cfm_model* m, const float* feats_dev, const int32_t* plan_host,
                                    const int32_t* plan_dev, const float* att_cache_in, const float* cnn_cache_in,
                                    int32_t truncated_context_size, float* att_cache_out, float* cnn_cache_out,
                                    float* out_dev, void* workspace, size_t workspace_bytes, int32_t stage_lo,
                                    int32_t stage_hi, cfm_stream stream);

/* cfm_encode_padded replaces ChunkFormerEncoder.forward_encoder (encoder.py:220-274)
 * and therefore ChunkFormerModel.encode (chunkformer_model.py:256-274).
 * xs_dev: [B, T, 80] f32 padded batch; out_dev: [B, T', d] f32. */
size_t cfm_workspace_bytes_padded(const cfm_model* m, int32_t B, int32_t T, int32_t chunk_size, int32_t left_context,
                                  int32_t right_context);
cfm_status cfm_encode_padded(const cfm_model* m, const float* xs_dev, const int32_t* plan_host, const int32_t* plan_dev,
                             float* out_dev, void* workspace, size_t workspace_bytes, cfm_stream stream);

/* ------------------------------------------------------------------ streaming
 * cfm_plan_stream + cfm_encode_stream replace ChunkFormerEncoder.forward_chunk
 * (encoder.py:310-385), the realtime path (apps/realtime-asr/stream_asr.py:164-172):
 * xs_dev [B, T, 80] f32 (every frame valid), T' = calc_length(T) with
 * right_context_size <= T' <= chunk_size + right_context_size; `offset` = frames already
 * streamed (keys of the first L - offset cache slots are masked, encoder.py:351-357).
 * att_cache_in [nb, B, H, L, 2*dk] and cnn_cache_in [nb, B, d, 7] f32 are required (the
 * reference's head-major layout); the new caches (encoder.py:374-383) go to
 * att_cache_out / cnn_cache_out (may alias the inputs; NULL = not wanted).  out_dev: [B, T', d]
 * f32 after after_norm.  One plan serves every batch element (they share T and offset). */
cfm_status cfm_plan_stream(int32_t T, int32_t chunk_size, int32_t left_context, int32_t right_context, int32_t offset,
                           int32_t* t_out, int32_t* plan_host, int64_t* plan_ints);
size_t cfm_workspace_bytes_stream(const cfm_model* m, int32_t T, int32_t chunk_size, int32_t left_context,
                                  int32_t right_context);
cfm_status cfm_encode_stream(const cfm_model* m, const float* xs_dev, int32_t B, const int32_t* plan_host,
                             const int32_t* plan_dev, const float* att_cache_in, const float* cnn_cache_in,
                             float* att_cache_out, float* cnn_cache_out, float* out_dev, void* workspace,
                             size_t workspace_bytes, cfm_stream stream);

/* Materialise att_mask [N, L+C+R] and mask_pad [N, C+14] (0/1 bytes) of a masked
 * plan: the exact tensors encoder.py:627-645 builds. */
cfm_status cfm_masks_from_plan(const int32_t* plan_host, const int32_t* plan_dev, uint8_t* att_mask_dev,
                               uint8_t* mask_pad_dev, cfm_stream stream);

/* ------------------------------------------------------------------ CTC head
 * CTC.log_softmax (ctc.py:73-81) + argmax (chunkformer_model.py:437-438, 526-527)
 * over enc_dev [rows, d].  logp_dev [rows, V] may be NULL (ids only: logits go to
 * the workspace); ids_dev [rows] int32 may be NULL. */
size_t cfm_ctc_workspace_bytes(const cfm_model* m, int32_t rows);
cfm_status cfm_ctc_logprobs(const cfm_model* m, const float* enc_dev, int32_t rows, float* logp_dev, int32_t* ids_dev,
                            void* workspace, size_t workspace_bytes, cfm_stream stream);

/* Fused CTC tail, ids only: ids_dev[rows] = argmax of CTC.log_softmax (ctc.py:73-81) as
 * chunkformer_model.py:437-438 / 526-527 take it.  On bf16 models with d_model 512 the logits never
 * leave registers (no [rows, V] tensor; workspace 0 bytes); otherwise it runs the log-softmax path
 * in the workspace (cfm_ctc_ids_workspace_bytes). */
size_t cfm_ctc_ids_workspace_bytes(const cfm_model* m, int32_t rows);
cfm_status cfm_ctc_ids(const cfm_model* m, const float* enc_dev, int32_t rows, int32_t* ids_dev, void* workspace,
                       size_t workspace_bytes, cfm_stream stream);

/* CTC post-processing on device, one utterance b = frames [row_start[b], row_start[b] + row_len[b])
 * of ids_dev (device int32 arrays; regions must not overlap).  Outputs are written compacted at
 * the start of each utterance's region:
 *   max_silence < 0: remove_duplicates_and_blank (utils/model_utils.py:23-32): tokens[] and the
 *     frame of each token (gen_ctc_peak_time, model_utils.py:49-58), n_tokens[b];
 *   max_silence >= 0: the sentence split of get_output_with_timestamps (model_utils.py:174-221)
 *     at max_silence (= max_silence_duration // 0.08) blank frames: per segment the de-duplicated
 *     non-blank tokens (tokens[], token_frames[]) and segments[s] = {first token, start frame,
 *     end frame} (80 ms frames), n_tokens[b], n_segments[b]. */
cfm_status cfm_ctc_collapse(const int32_t* ids_dev, const int32_t* row_start_dev, const int32_t* row_len_dev, int32_t B,
                            int32_t blank_id, int32_t max_silence, int32_t* tokens_dev, int32_t* token_frames_dev,
                            int32_t* n_tokens_dev, int32_t* segments_dev /* [rows, 3] or NULL */,
                            int32_t* n_segments_dev /* [B] or NULL */, cfm_stream stream);

/* ---- Kaldi log-mel filterbank (the reference's feature front: chunkformer_model.py:276-318 and
 * dataset/processor.py:210-239 call torchaudio.compliance.kaldi.fbank).  Fields and defaults follow
 * torchaudio's fbank() signature; the reference decodes with dither 0, energy_floor 0, 80 bins,
 * 25 / 10 ms, povey window, int16-scale samples.  Supported: dither 0, snip_edges, use_energy 0,
 * padded frames of 128 .. 1024 samples. */
typedef enum { CFM_WINDOW_POVEY = 0, CFM_WINDOW_HAMMING = 1, CFM_WINDOW_HANNING = 2, CFM_WINDOW_RECTANGULAR = 3,
               CFM_WINDOW_BLACKMAN = 4 } cfm_window_type;
typedef struct {
  float sample_frequency;        /* 16000 */
  float frame_length_ms;         /* 25 */
  float frame_shift_ms;          /* 10 */
  int32_t num_mel_bins;          /* 80 in the reference (torchaudio default 23) */
  float low_freq;                /* 20 */
  float high_freq;               /* 0: Nyquist; < 0: offset from Nyquist */
  float preemphasis_coefficient; /* 0.97 */
  float dither;                  /* must be 0 */
  int32_t remove_dc_offset;      /* 1 */
  int32_t round_to_power_of_two; /* 1 */
  int32_t snip_edges;            /* must be 1 */
  int32_t use_energy;            /* must be 0 */
  int32_t use_log_fbank;         /* 1 */
  int32_t window_type;           /* cfm_window_type, POVEY (blackman uses coefficient 0.42) */
} cfm_fbank_config;
typedef struct cfm_fbank cfm_fbank;

/* window, FFT twiddles and mel filters on `device` (replaces the per-call get_mel_banks /
 * _feature_window_function of compliance/kaldi.py) */
cfm_status cfm_fbank_create(const cfm_fbank_config* cfg, int32_t device, cfm_fbank** out);
void cfm_fbank_destroy(cfm_fbank* h);
/* frames of a waveform of num_samples samples: 1 + (n - win) / shift, 0 when n < win */
int64_t cfm_fbank_num_frames(const cfm_fbank* h, int64_t num_samples);
/* out_dev[frames, num_mel_bins] (f32) = kaldi.fbank(wave_dev[num_samples]) (f32 device samples,
 * int16 scale); stream-ordered, no allocation, no host synchronisation */
cfm_status cfm_fbank_compute(const cfm_fbank* h, const float* wave_dev, int64_t num_samples, float* out_dev,
                             cfm_stream stream);

/* ---- RNN-T consumer (model: transducer checkpoints): greedy search over encoder outputs, the
 * reference's optimized_search / batch_greedy_search (transducer/search/greedy_search.py:6-92) as
 * endless_decode / batch_decode call them (chunkformer_model.py:439-448, 533-543), with the shipped
 * RNNPredictor (lstm; transducer/predictor.py:66-208) and TransducerJoint (prejoin_linear, add,
 * tanh, ffn_out; transducer/joint.py:74-111).  Predictor and joint compute in f32. */
typedef struct {
  int32_t vocab;        /* output_dim */
  int32_t enc_dim;      /* joint_conf.enc_output_size (the encoder's d_model) */
  int32_t embed_size;   /* predictor_conf.embed_size */
  int32_t hidden;       /* predictor_conf.hidden_size */
  int32_t num_layers;   /* predictor_conf.num_layers (<= 4) */
  int32_t pred_out;     /* predictor_conf.output_size = joint_conf.pred_output_size */
  int32_t join_dim;     /* joint_conf.join_dim */
  int32_t blank;        /* 0 (init_model.py:125-128) */
} cfm_rnnt_config;
typedef struct cfm_rnnt cfm_rnnt;

/* weights by reference key: predictor.embed.weight, predictor.rnn.{weight,bias}_{ih,hh}_l{k},
 * predictor.projection.{weight,bias}, joint.{enc_ffn,pred_ffn,ffn_out}.{weight,bias} */
cfm_status cfm_rnnt_create(const cfm_rnnt_config* cfg, const cfm_tensor_view* weights, int32_t n_weights,
                           int32_t device, cfm_rnnt** out);
void cfm_rnnt_destroy(cfm_rnnt* h);
size_t cfm_rnnt_workspace_bytes(const cfm_rnnt* h, int32_t rows);
/* Greedy search of utterances b = rows [row_start[b], row_start[b] + row_len[b]) of enc_dev
 * [rows, enc_dim] f32 (device int32 row arrays).  out_dev [rows, n_steps] int32 must be zeroed by the
 * caller; row t of an utterance receives the ids decided at its frame t in step order, exactly the
 * reference's output[:, t * n_steps + step] with the sos column removed (0 = blank). */
cfm_status cfm_rnnt_greedy(const cfm_rnnt* h, const float* enc_dev, int32_t rows, const int32_t* row_start_dev,
                           const int32_t* row_len_dev, int32_t B, int32_t n_steps, int32_t* out_dev, void* workspace,
                           size_t workspace_bytes, cfm_stream stream);
/* cfm_rnnt_greedy with per-call flags: CFM_RNNT_ONE_WORKGROUP runs this call on the one-workgroup kernel
 * whatever "grid_blocks" says (the caller's rerun after a grid barrier timed out), leaving the handle's
 * options and its grid weight image untouched. */
#define CFM_RNNT_ONE_WORKGROUP 1
cfm_status cfm_rnnt_greedy_ex(const cfm_rnnt* h, const float* enc_dev, int32_t rows, const int32_t* row_start_dev,
                              const int32_t* row_len_dev, int32_t B, int32_t n_steps, int32_t* out_dev, void* workspace,
                              size_t workspace_bytes, int32_t flags, cfm_stream stream);
/* Options: "grid_lds" (default 1) caches each workgroup's weight slices in LDS when they fit;
 * "grid_atomic" (default 1) exchanges the shared vectors by agent-scope atomics instead of fences;
 * "grid_blocks" = workgroups per utterance of the multi-CU search (default 32; 0 = one
 * workgroup per utterance always).  The multi-CU search runs when B <= 32 and B * grid_blocks <= the
 * device's CU count; cfm_rnnt_grid_blocks returns the workgroups per utterance a call with B
 * utterances uses (0: the one-workgroup kernel). */
cfm_status cfm_rnnt_set_option(cfm_rnnt* h, const char* key, int64_t value);
int32_t cfm_rnnt_grid_blocks(const cfm_rnnt* h, int32_t B);
/* After a multi-CU call has completed: nonzero if one of its grid barriers timed out (the search then
 * stopped early and its output is incomplete); -1 if the word could not be read.  Synchronous. */
int32_t cfm_rnnt_error(const cfm_rnnt* h, const void* workspace, int32_t rows);

#ifdef __cplusplus
}
#endif
#endif /* CFM_H */
