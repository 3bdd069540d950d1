/*
 * wakeword_host.h -- C ABI of libwakeword_host.so: the same wake-word path on
 * the HOST CPU, for callers without a GPU (BASELINE config 1, "single WAV on
 * CPU") and for firmware-side code that links mfcc.c's interface.
 *
 * This is a separate library, not a fallback inside libwakeword.so: the GPU
 * library never calls it, and it never touches HIP.  A caller chooses it by
 * linking / loading it (Python: wakeword.host, `python -m wakeword.test --cpu`).
 * Everything is plain C: host pointers, sizes, wk_status codes (wakeword.h).
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   - main/esp_mfcc/mfcc.h:10-17, mfcc.c:298-299  extract_mfcc / free_mfcc /
 *     analyze_mfcc_range / flow_extract_mfcc_single_frame: host code there,
 *     host code here, same signatures, ownership and NULL-on-error behaviour
 *     (mfcc.c:431-527, :297-427, :530-563)
 *   - ml_models/src/extract_mfcc.py:137-175 + :47-88  MFCC (torchaudio
 *     definition) + normalize_mfcc('cmvn')                       (wkh_mfcc)
 *   - ml_models/src/wakeModel.py:29-34  LightweightKWS.forward     (wkh_cnn)
 *   - ml_models/test.py / main.py:52-53 WAV -> features -> logit   (wkh_forward)
 *
 * Threads: batch calls split their clips over wkh_set_threads() host threads
 * (default: the hardware concurrency).  Calls on distinct models and the
 * stateless functions are thread-safe; the mfcc.h functions are too (unlike
 * mfcc.c's static tables, every table here is built per call or cached under
 * a lock).
 */
#ifndef WAKEWORD_HOST_H_
#define WAKEWORD_HOST_H_

#include "wakeword.h"   /* wk_status, WK_NUM_WEIGHTS, and the mfcc.h prototypes this library also exports */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wkh_model wkh_model;

/* A host model from the WK_NUM_WEIGHTS packed weights wk_create() takes
 * (conv_layers.{0,3,6}.weight, classifier.{0,2}.weight, state-dict layouts). */
wk_status wkh_create(const float* weights, wkh_model** out);
wk_status wkh_destroy(wkh_model* m);

/* Mode B front-end (extract_mfcc.py:137-175): batch clips of win_len == 16000
 * samples (clip i at audio + i*stride) -> feats[batch][13][63]; cmvn = 1 applies
 * normalize_mfcc('cmvn') (the training path), 0 leaves raw MFCC. */
wk_status wkh_mfcc(const float* audio, int64_t batch, int32_t win_len, int64_t stride, int32_t cmvn, float* feats);

/* LightweightKWS.forward on given features [batch][13][63] -> logits[batch]. */
wk_status wkh_cnn(const wkh_model* m, const float* feats, int64_t batch, float* logits);

/* Audio -> CMVN'd mode-B features -> CNN -> logits[batch] (feats_or_null: also
 * the features, [batch][13][63]). */
wk_status wkh_forward(const wkh_model* m, const float* audio, int64_t batch, int32_t win_len, int64_t stride,
                      float* logits, float* feats_or_null);

/* Mode A (mfcc.c) at any parameter set in its domain (n_fft a power of two in
 * [2, 4096], 1 <= n_filters <= 1024, frame_size, n_mfcc, sampling_rate >= 1):
 * batch signals of signal_len samples -> out[batch][n_frames][n_mfcc],
 * n_frames = (signal_len - frame_size) / hop_size + 1; pre_emphasis 0.97 as
 * extract_mfcc, 0 as the single-frame variant. */
wk_status wkh_esp_mfcc(const float* signal, int64_t batch, int32_t signal_len, int64_t stride, int32_t sampling_rate,
                       int32_t frame_size, int32_t hop_size, int32_t n_fft, int32_t n_filters, int32_t n_mfcc,
                       int32_t esp_dsp_packing, float pre_emphasis, float* out);

/* Host threads for batch calls (n >= 1; 0 = the hardware concurrency).  Returns the value in effect. */
int32_t wkh_set_threads(int32_t n);
const char* wkh_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* WAKEWORD_HOST_H_ */
