/*
 * wakeword.h -- C ABI of the MI355X (gfx950) wake-word inference path.
 *
 * Drop-in boundary for the reference's hot path (Socrates666/esp32-wake-word):
 *   audio window -> MFCC front-end -> xiaoa CNN (LightweightKWS) -> logit.
 * Everything here is plain C: pointers, sizes, status codes; no C++ or torch
 * types cross the boundary.  Device pointers are HIP device memory; `stream`
 * is a hipStream_t passed as void* (NULL = the legacy default stream).
 * Calls that take device pointers are stream-ordered, allocate nothing and
 * never block the host.  Errors are reported as wk_status codes, never aborts.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   - main/esp_mfcc/mfcc.h:10-17   extract_mfcc / free_mfcc / analyze_mfcc_range
 *                                  (identical signatures and ownership below)
 *   - ml_models/src/wakeModel.py:29-34  LightweightKWS.forward (wk_cnn)
 *   - ml_models/src/extract_mfcc.py:137-175  MFCC + CMVN front-end (wk_mfcc)
 *   - main/hello_world_main.cpp:183-267 / esp_wake_word_detector.cpp:154-228
 *     per-window MFCC -> model->run() -> sigmoid (wk_forward)
 */
#ifndef WAKEWORD_H_
#define WAKEWORD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WK_ABI_VERSION 1

typedef enum {
  WK_OK = 0,
  WK_ERR_INVALID_ARG = 1,   /* null pointer, bad size, unsupported parameter combo */
  WK_ERR_HIP = 2,           /* a HIP runtime call failed (see wk_last_error())     */
  WK_ERR_NO_MEMORY = 3,     /* device or host allocation failed                    */
  WK_ERR_UNSUPPORTED = 4,   /* valid request this build does not implement         */
  WK_ERR_DEVICE = 5         /* a kernel reported an internal protocol failure: the */
                            /* results of the launches it covers are invalid       */
} wk_status;

/* Front-end definitions. */
typedef enum {
  WK_MODE_TORCHAUDIO_CMVN = 0, /* mode B: extract_mfcc.py:137-175 (+ CMVN), out [13][63] */
  WK_MODE_ESP_MFCC = 1         /* mode A: esp_mfcc/mfcc.c:431-527, out [n_frames][13]     */
} wk_mode;

typedef enum { WK_DTYPE_F32 = 0, WK_DTYPE_I16 = 1, WK_DTYPE_I8 = 2 } wk_dtype;   /* sample / frame type */
/* CNN arithmetic.  FP32 = fp32 MFMA.  BF16 = bf16 convolutions (SURVEY
 * config 4), fp32 front-end/classifier.  INT8 = the device's esp-dl int8
 * network (power-of-2 per-tensor exponents of ml_models/xiaoa.info,
 * round-half-even requant; reproduces the xiaoa.info known-answer test
 * exactly): a device-faithful checking mode, run unfused after the fp32
 * front-end.  BF16X3 = fp32-grade convolutions on bf16 MFMA: activations and
 * weights split into bf16 hi + lo parts, products hi*hi + hi*lo + lo*hi
 * accumulated in fp32 (relative product error ~2^-16); same logit tolerance
 * as FP32.  Every precision runs in wk_forward and in wk_cnn. */
typedef enum { WK_PREC_FP32 = 0, WK_PREC_BF16 = 1, WK_PREC_INT8 = 2, WK_PREC_BF16X3 = 3 } wk_precision;

typedef struct {
  int32_t mode;            /* wk_mode                                               */
  int32_t precision;       /* wk_precision (front-end is always fp32)               */
  int32_t esp_dsp_packing; /* mode A only: 1 = emulate dsps_cplx2reC_fc32 packing    */
  int32_t device;          /* HIP device ordinal the handle binds to                */
  int32_t cmvn;            /* mode B only: 1 = normalize_mfcc('cmvn') (the training */
                           /* path, extract_mfcc.py:175), 0 = raw MFCC              */
} wk_config;

typedef struct wk_handle wk_handle;

/* Number of floats in the packed weight blob wk_create() expects:
 * conv_layers.0.weight [32][13][3], conv_layers.3.weight [64][32][3],
 * conv_layers.6.weight [128][64][3], classifier.0.weight [64][128],
 * classifier.2.weight [1][64] -- PyTorch state-dict layouts, concatenated. */
#define WK_NUM_WEIGHTS 40224

/* Fixed geometry of the xiaoa model (1 s @ 16 kHz). */
#define WK_WIN_SAMPLES 16000
#define WK_N_MFCC 13
#define WK_N_FRAMES_B 63

/* Create a handle on cfg->device.  `host_weights` (WK_NUM_WEIGHTS floats, host
 * memory) may be NULL for a front-end-only handle.  Replaces the reference's
 * `new dl::Model(...)` + weight load (hello_world_main.cpp:178). */
wk_status wk_create(const wk_config* cfg, const float* host_weights, wk_handle** out);
wk_status wk_destroy(wk_handle* h);

/* The fused kernel's two roles (front-end waves, CNN waves) hand clips over
 * through bounded spins, and the CNN role's waves (also behind wk_cnn)
 * synchronise through bounded spins; a spin that times out (a protocol
 * failure -- never expected) ends the launch with invalid logits instead of a
 * hung GPU, and raises a flag in a host-visible word of the handle.  This call synchronises
 * the handle's device, returns WK_ERR_DEVICE if any launch on the handle since
 * the last check raised it (flags in *flags_out, may be NULL; 0 = clean), and
 * clears it.  A wk_stream has its own word (its pushes' launches report there,
 * not to the handle's): wk_stream_push checks and clears it on every push. */
wk_status wk_check_device_errors(wk_handle* h, uint32_t* flags_out);

/* Front-end only.  d_audio: `batch` clips of `win_len` samples, clip i at
 * d_audio + i*clip_stride elements (dtype WK_DTYPE_F32 or WK_DTYPE_I16; i16 is
 * scaled by 1/32768 like torchaudio.load).  Mode B requires win_len == 16000
 * and writes CMVN'd features [batch][13][63]; mode A accepts win_len >= 320
 * (clip_stride may be smaller than win_len: overlapping sliding windows)
 * and writes [batch][n_frames][13] with n_frames = (win_len-320)/256+1. */
wk_status wk_mfcc(wk_handle* h, const void* d_audio, int32_t dtype, int64_t batch, int32_t win_len,
                  int64_t clip_stride, float* d_feats, void* stream);

/* CNN only: d_feats [batch][13][63] -> d_logits [batch] (LightweightKWS.forward). */
wk_status wk_cnn(wk_handle* h, const float* d_feats, int64_t batch, float* d_logits, void* stream);

/* Fused hot path: audio -> logits [batch]; mode B only (the model's training
 * front-end).  d_feats_or_null, when given, receives the [batch][13][63]
 * features as well.  A handle may be used from several streams and host
 * threads: the INT8 / unfused path stages features in a per-handle workspace
 * (when d_feats_or_null is NULL) and orders its uses across streams with an
 * event; the fused path shares nothing between calls. */
wk_status wk_forward(wk_handle* h, const void* d_audio, int32_t dtype, int64_t batch, int32_t win_len,
                     int64_t clip_stride, float* d_logits, float* d_feats_or_null, void* stream);

/* Device-side synthetic clip generator: fills
 * d_out[count][n] with clips first..first+count-1 of the counter-based
 * generator keyed on `seed` (bit-compatible with oracle.synth_clips up to
 * libm rounding). */
wk_status wk_synth_clips(uint32_t seed, int64_t first, int64_t count, int32_t n, float* d_out, void* stream);

/* normalize_mfcc(mfcc, method) (extract_mfcc.py:47-88) on device:
 * d_in/d_out [batch][n_coef][n_time]; method 0 = 'standardization',
 * 1 = 'minmax', 2 = 'cmvn', 3 = passthrough. In-place allowed. */
wk_status wk_normalize(const float* d_in, float* d_out, int64_t batch, int32_t n_coef, int32_t n_time,
                       int32_t method, void* stream);

/* ---- Streaming -------------------------------------
 * A device ring of `capacity` samples (>= 16000 + hop) fed from host memory,
 * with ring_buffer.c:57-117's overwrite-oldest semantics (write_rinbuffer).
 * Window k covers stream samples [k*hop, k*hop + 16000) -- the device's
 * continuously re-scored 1 s window (esp_wake_word_detector.cpp:52-150 slides
 * it frame by frame).  wk_stream_push() appends n float samples, scores every
 * window the push completes (oldest first; windows whose start was already
 * overwritten are dropped, and when more than max_out complete only the
 * newest max_out are scored) with the fused path on the handle's device, and
 * returns their logits and end positions (samples since create/reset) in host
 * memory.  It blocks until the logits are on the host.  Not thread-safe per
 * stream object.  The ring lives in device memory behind a pinned host
 * staging ring; a push that completes windows is two launches and one wait:
 * a small kernel reads the samples pushed since the last such push across
 * PCIe into the device ring, then the fused kernel scores the windows from
 * HBM and writes the logits to pinned host memory (no copy commands). */
typedef struct wk_stream wk_stream;
wk_status wk_stream_create(wk_handle* h, int32_t hop, int32_t capacity, void* stream, wk_stream** out);
wk_status wk_stream_destroy(wk_stream* s);
wk_status wk_stream_reset(wk_stream* s);   /* forget history (post-detection reset, detector.cpp:249-256) */
wk_status wk_stream_push(wk_stream* s, const float* host_samples, int64_t n, float* out_logits, int64_t* out_end,
                         int32_t max_out, int32_t* n_out);

/* ---- The firmware's detector over an MFCC frame stream --
 * esp_wake_word_detector.cpp keeps the last 63 int8 MFCC frames of 13
 * coefficients (record_task :128-134 quantises each 20 ms frame with lroundf +
 * saturation; write_one_frame_mfcc_to_buffer / read_whole_mfcc_buffer :21-48
 * hand the detector the 63 newest frames, oldest first) and, per window,
 * applies its own CMVN (detect_task :179-211: mean and POPULATION std over the 63
 * frames, (v - mean) / (std + 1e-8), lroundf, saturate) before the int8 model.
 * wk_device_cmvn runs that CMVN for every window of a frame stream: d_frames
 * [n_frames][13] (WK_DTYPE_I8 = the firmware's int8 frames, or WK_DTYPE_F32 =
 * float MFCC frames, quantised first as record_task does); window w = frames
 * w .. w+62, n_frames - 62 windows (none if n_frames < 63).  Outputs (either may
 * be NULL, not both): d_out_i8 [w][63][13] -- the firmware's mfcc_cmvn_buffer --
 * and d_feats_or_null [w][13][63], the same integer values as floats in wk_cnn's
 * layout (feed it to a WK_PREC_INT8 handle for the device's int8 network:
 * dl::TensorBase::assign from exponent 0 to the input exponent -4 is x16 with
 * saturation, which is what WK_PREC_INT8 applies to its float input).
 * Bit-identical to the firmware's C loops (same fp32 summation order). */
wk_status wk_device_cmvn(const void* d_frames, int32_t dtype, int64_t n_frames, int8_t* d_out_i8,
                         float* d_feats_or_null, void* stream);

/* ---- The firmware record task's front (esp_wake_word_detector.cpp:52-150) ---
 * wk_record_front: the sample path of record_task (:102-121), integer-exact.
 * d_tdm holds 3*n_out 48 kHz TDM samples of 4 int16 channels (interleaved
 * CH0 MIC-L, CH1 AEC reference, CH2 MIC-R, CH3 unused; the firmware reads 960
 * of them = 3840 int16 per 20 ms frame); per TDM sample the mono mix
 * m = (int16_t)(((L<<6) + (AEC<<5) + (R<<6)) >> 7) keeps the low 16 bits of the
 * int32 sum as the firmware's cast does; then d_out16[j] =
 * (int16_t)((m[3j] + 2 m[3j+1] + m[3j+2]) >> 2) at 16 kHz (320 per frame).
 * Frames are independent of each other (960 = 3 x 320), so any run of frames
 * is one call.  d_out_f32_or_null receives d_out16 / 32768.  d_out16 can feed
 * wk_forward directly as WK_DTYPE_I16 (clip_stride = hop: sliding windows);
 * the esp-dl MFCC the firmware runs on it (:124-125) is third-party and absent.
 * Alignment: d_tdm 16 bytes, d_out16 4, d_out_f32 8. */
wk_status wk_record_front(const int16_t* d_tdm, int64_t n_out, int16_t* d_out16, float* d_out_f32_or_null,
                          void* stream);
/* record_task's frame quantisation (:128-131): d_out_i8[i] = saturate_int8(lroundf(d_mfcc[i])),
 * n_values = 13 x frames; the result feeds wk_device_cmvn as WK_DTYPE_I8. */
wk_status wk_quantize_frames(const float* d_mfcc, int64_t n_values, int8_t* d_out_i8, void* stream);

/* ---- CTC head (ml_models/ctc.py) -------------------------
 * GRU_CTC_Model (ctc.py:119-152) + its log-mel front-end (ctc.py:82-107) +
 * greedy decode (ctc.py:453-471).  The reference builds V from its corpus at
 * run time (ctc.py:261-278); here V is a parameter.  This build implements the
 * reference Config (ctc.py:21-40): hidden 128, 2 bidirectional GRU layers,
 * 80 mels, n_fft 400, hop 160.  A wk_ctc handle owns its activations
 * workspace: issue one handle's calls on one stream (or order them across
 * streams yourself); use one handle per stream for concurrent batches. */
typedef struct {
  int32_t vocab;    /* V, including <blank> = 0 and <unk> = 1                */
  int32_t hidden;   /* 128 */
  int32_t layers;   /* 2 */
  int32_t n_mels;   /* 80 */
  int32_t device;
  int32_t precision; /* 0: fp32 throughout; 1 (config 5 "fp16"): GEMM and
                        MFMA operands, activations between layers and the gate
                        pre-activations in fp16, fp32 accumulation; the gate
                        arithmetic, state update and front-end stay fp32 */
} wk_ctc_config;
typedef struct wk_ctc wk_ctc;

/* Floats in the weight blob: the GRU_CTC_Model state dict in its own order
 * (audio_encoder.{0,1}.{weight,bias}, gru.{weight_ih,weight_hh,bias_ih,bias_hh}
 * _l{0,1}[_reverse], output_layer.{weight,bias}), concatenated. */
int64_t wk_ctc_num_weights(const wk_ctc_config* cfg);
wk_status wk_ctc_create(const wk_ctc_config* cfg, const float* host_weights, wk_ctc** out);
wk_status wk_ctc_destroy(wk_ctc* c);
/* X1 extract_features: d_audio [batch] rows of float samples (row i at
 * d_audio + i*stride, n_valid samples each) zero-padded / trimmed to
 * n_samples (ctc.py:85-90, max_audio_length) -> d_feats [batch][T][80],
 * T = 1 + n_samples/160, ln(mel+1e-8) z-scored per utterance (ctc.py:95-104). */
wk_status wk_ctc_features(wk_ctc* c, const float* d_audio, int64_t batch, int32_t n_valid, int32_t n_samples,
                          int64_t stride, float* d_feats, void* stream);
/* X2 + X3: d_feats [batch][T][80] -> greedy CTC tokens d_tokens [batch][T]
 * (blank-free, repeats collapsed, padded with -1) and d_lengths [batch];
 * d_log_probs_or_null [batch][T][V] receives log_softmax when given.  The
 * handle's workspace grows on the first call with a larger batch*T. */
wk_status wk_ctc_forward(wk_ctc* c, const float* d_feats, int64_t batch, int32_t T, float* d_log_probs_or_null,
                         int32_t* d_tokens, int32_t* d_lengths, void* stream);

/* X1 + X2 + X3 in one call (audio -> greedy tokens): the same result as
 * wk_ctc_features into a handle-owned buffer followed by wk_ctc_forward
 * without log-probs (ctc.py:82-107 then :148-152, :453-471).  In fp16 mode
 * (precision 1) with T >= 6 the z-score is not applied in place: the log-mel
 * kernel also leaves per-pass sums, a small kernel turns them into each
 * utterance's mean and 1/std, and the encoder applies them as it loads the
 * raw rows -- one read and one write of the [batch][T][80] features fewer.
 * The statistics then differ from wk_ctc_features' by float rounding, so a
 * token may differ only where two logits are within that noise.  An
 * utterance whose log-mel values are all equal (digital silence) is left
 * un-normalised (std = 0 exactly).  Workspace grows on first use. */
wk_status wk_ctc_transcribe(wk_ctc* c, const float* d_audio, int64_t batch, int32_t n_valid, int32_t n_samples,
                            int64_t stride, int32_t* d_tokens, int32_t* d_lengths, void* stream);

/* Stage timing for measurement (bench_ctc.py): while enabled, every stage of
 * wk_ctc_features / wk_ctc_forward is bracketed by a pair of HIP events on the
 * call's stream; wk_ctc_stage_times synchronises on them and returns, per
 * stage, the summed milliseconds and the number of timed launches since the
 * last wk_ctc_profile call (which clears them).  Off by default (no events). */
enum {
  WK_CTC_STAGE_LOGMEL = 0,  /* X1 log-mel (framing, FFT, power, mel, ln)            */
  WK_CTC_STAGE_ZSCORE,      /* X1 global z-score (wk_ctc_transcribe fp16: its statistics only) */
  WK_CTC_STAGE_ENCODER,     /* Linear 80->128 + LayerNorm + ReLU                    */
  WK_CTC_STAGE_PROJ0,       /* GRU layer 0 input projection (x W_ih^T, both dirs)   */
  WK_CTC_STAGE_GRU0,        /* GRU layer 0 recurrence (both directions)             */
  WK_CTC_STAGE_PROJ1,       /* GRU layer 1 input projection                         */
  WK_CTC_STAGE_GRU1,        /* GRU layer 1 recurrence                               */
  WK_CTC_STAGE_OUTPUT,      /* output layer + argmax (+ log_softmax when requested) */
  WK_CTC_STAGE_DECODE,      /* greedy CTC collapse                                  */
  WK_CTC_N_STAGES
};
wk_status wk_ctc_profile(wk_ctc* c, int32_t enable);
wk_status wk_ctc_stage_times(wk_ctc* c, double* ms_sum /* [WK_CTC_N_STAGES] */, int64_t* counts /* [WK_CTC_N_STAGES] */);

/* X3's per-frame argmax -- decode_predictions' `predictions` (ctc.py:454,
 * first maximum per frame), the frame tokens the greedy decode collapsed --
 * of the handle's last wk_ctc_forward: d_pred [batch][T] int32.  batch and T
 * must be that call's (else WK_ERR_INVALID_ARG); stream-ordered after it. */
wk_status wk_ctc_frame_argmax(wk_ctc* c, int64_t batch, int32_t T, int32_t* d_pred, void* stream);

/* ---- WAV ingest and waveform augmentation (host only) ---
 * No device work: these fill caller (e.g. pinned) host buffers for the H2D copy. */
typedef struct {
  int32_t sample_rate, channels, bits_per_sample;
  int32_t data_samples;   /* frames in the data chunk              */
  int32_t n_samples;      /* frames actually read (<= max_samples) */
} wk_wav_info;
/* esp_wav.cpp:8-139: RIFF/WAVE/"fmt " header, unknown chunks before "data"
 * skipped, PCM 16-bit only (WK_ERR_UNSUPPORTED otherwise); channel 0 of up
 * to max_samples frames into out (the reference truncates to 16000). */
wk_status wk_wav_read(const char* path, int16_t* out, int32_t max_samples, wk_wav_info* info);
/* torchaudio.load scaling (x/32768) + pad_audio (extract_mfcc.py:7-23) for n
 * files on worker threads: out[n][pad_to], right-padded with N(0,
 * noise_level^2) from a counter-hash generator keyed on (seed, file index)
 * (distribution of torch.randn * noise_level, not its bit stream), or zeros
 * when noise_level == 0.  n_read[i] (may be NULL) gets each file's length. */
wk_status wk_wav_load_batch(const char* const* paths, int32_t n, int32_t pad_to, float noise_level, uint32_t seed,
                            float* out, int32_t* n_read);
/* augment_audio_waveform (extract_mfcc.py:90-121): speed change by linear
 * interpolation to int(n*speed) samples (F.interpolate, align_corners=False),
 * padded (noise as above, stream 0) / trimmed to out_len, then x volume with
 * clamp to [-1, 1] when volume != 1. */
wk_status wk_augment(const float* in, int32_t n, float speed, float volume, float noise_level, uint32_t seed, float* out,
                     int32_t out_len);

/* Human-readable text for a status / the last HIP error seen by this thread. */
const char* wk_status_string(wk_status s);
const char* wk_last_error(void);
int32_t wk_abi_version(void);

/* ---- mode A at any parameter set (main/esp_mfcc/mfcc.c:144-234,298-527) ----
 * mfcc.c accepts any sampling rate, frame, hop, n_fft, n_filters and n_mfcc
 * and rebuilds its filterbank, window and DCT tables per call.  A
 * wk_esp_mfcc object holds one parameter set's tables on `device` (built
 * with the reference's float formulas); wk_esp_mfcc_run computes, on the
 * GPU, batch signals of signal_len samples (signal i at d_signal + i*stride)
 * -> d_out[batch][n_frames][n_mfcc], n_frames = (signal_len - frame_size) /
 * hop_size + 1: pre-emphasis `pre_emphasis` (0.97 in extract_mfcc, 0 in the
 * single-frame variant), symmetric Hamming (alpha 0.53836), the frame in the
 * first min(frame_size, n_fft) points of an n_fft-point FFT, power /n_fft +
 * 1e-12 (esp_dsp_packing: dsps_cplx2reC_fc32's packing), mel, ln(max(E,1e-12)),
 * DCT-II; coefficients past n_filters are 0 (mfcc.c's calloc).
 * Domain: n_fft a power of two in [2, 4096] (esp-dsp's FFT refuses other
 * lengths), 1 <= n_filters <= 1024, frame_size, n_mfcc, sampling_rate >= 1;
 * WK_ERR_INVALID_ARG outside it. */
typedef struct wk_esp_mfcc wk_esp_mfcc;
wk_status wk_esp_mfcc_create(int32_t sampling_rate, int32_t frame_size, int32_t n_fft, int32_t n_filters,
                             int32_t n_mfcc, int32_t esp_dsp_packing, int32_t device, wk_esp_mfcc** out);
wk_status wk_esp_mfcc_run(wk_esp_mfcc* m, const float* d_signal, int64_t batch, int32_t signal_len, int64_t stride,
                          int32_t hop_size, float pre_emphasis, float* d_out, void* stream);
wk_status wk_esp_mfcc_destroy(wk_esp_mfcc* m);

/* ---- mfcc.h compatibility shims (main/esp_mfcc/mfcc.h:10-17) --------------
 * Same signatures and ownership as the reference: host signal in, a malloc'd
 * host block of n_frames*n_mfcc floats (frame-major) out, caller frees it with
 * free_mfcc(); NULL on bad arguments.  Computed on device 0 with
 * esp_dsp_packing on: the reference configuration (16000 Hz, 320/256/512, 40
 * filters, 13 coefficients) by the fixed-geometry mode-A kernel, every other
 * parameter set in wk_esp_mfcc's domain by wk_esp_mfcc (tables cached per
 * parameter set); NULL outside that domain (non-power-of-2 n_fft, hop_size
 * < 1, ...). */
float* extract_mfcc(const float* signal, int signal_len, int sampling_rate, int frame_size, int hop_size,
                    int n_fft, int n_filters, int n_mfcc);
void free_mfcc(float* mfcc);
void analyze_mfcc_range(float* mfcc, int size, const char* label);
/* mfcc.c:297-427 (defined there, not declared in mfcc.h): one frame of
 * frame_size <= n_fft samples, no pre-emphasis -> malloc'd n_mfcc floats, NULL
 * on error. */
float* flow_extract_mfcc_single_frame(const float* frame, int frame_size, int sampling_rate, int n_fft, int n_filters,
                                      int n_mfcc);

#ifdef __cplusplus
}
#endif

#endif /* WAKEWORD_H_ */
