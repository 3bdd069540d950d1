// wk_kernels.h -- host-side launchers of the wake-word kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wk {

// Front-end (wk_frontend.hip).  mode_b: torchaudio+CMVN -> [B][13][63];
// otherwise esp_mfcc -> [B][n_frames][13].
hipError_t launch_frontend(bool mode_b, bool i16, const void* audio, int64_t batch, int win_len,
                           int64_t clip_stride, float* out, int esp_pack, int cmvn, int grid_cap,
                           hipStream_t stream);

// CNN (wk_cnn.hip): feats [B][13][63] -> logits [B].  `w` = device weight
// blob in the packed WK_NUM_WEIGHTS layout of include/wakeword.h.
hipError_t launch_cnn(const float* feats, int64_t batch, const float* w, float* logits, bool bf16,
                      int grid_cap, hipStream_t stream);

// Fused front-end + CNN (wk_fused.hip), mode B only.
hipError_t launch_fused(bool i16, const void* audio, int64_t batch, int64_t clip_stride, const float* w,
                        float* logits, float* feats_or_null, int grid_cap, hipStream_t stream);

// Misc (wk_misc.hip).
hipError_t launch_synth(uint32_t seed, int64_t first, int64_t count, int n, float* out, hipStream_t stream);
hipError_t launch_normalize(const float* in, float* out, int64_t batch, int n_coef, int n_time, int method,
                            hipStream_t stream);

// Offsets (floats) of each tensor inside the packed weight blob.
constexpr int kOffW1 = 0;                       // conv_layers.0.weight [32][13][3]
constexpr int kOffW2 = kOffW1 + 32 * 13 * 3;    // conv_layers.3.weight [64][32][3]
constexpr int kOffW3 = kOffW2 + 64 * 32 * 3;    // conv_layers.6.weight [128][64][3]
constexpr int kOffF1 = kOffW3 + 128 * 64 * 3;   // classifier.0.weight [64][128]
constexpr int kOffF2 = kOffF1 + 64 * 128;       // classifier.2.weight [1][64]
constexpr int kNumWeights = kOffF2 + 64;        // 40224

}  // namespace wk
