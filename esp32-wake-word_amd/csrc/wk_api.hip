// wk_api.hip -- the C ABI of include/wakeword.h.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include <mutex>
#include <new>
#include <vector>
#include <string>

#include "wakeword.h"
#include "wk_kernels.h"

struct wk_handle {
  wk_config cfg;
  int n_cu;
  unsigned* h_err;       // protocol error word of the fused kernel: pinned, mapped host memory ...
  unsigned* d_err;       // ... and its device alias (the kernel writes it, the host reads it after a sync)
  // The unfused / int8 path stages features in d_feats_ws.  Calls may come on
  // different streams (and host threads), so each use of the workspace waits
  // on the event recorded after the previous one (stream order across streams).
  std::mutex ws_mu;
  hipEvent_t ws_free;
  bool ws_used;
  bool ws_poisoned;      // the workspace's last use could neither be recorded nor drained: later
                         // staged forwards refuse to run (WK_ERR_HIP) rather than race it
  float* d_weights;      // packed WK_NUM_WEIGHTS floats, or nullptr (front-end only handle)
  float* d_packed;       // fragment-major weights (wk::pack_fragments) for the fused kernel
  float* d_feats_ws;     // feature workspace for the unfused path
  int8_t* d_int8;        // int8 weights (WK_PREC_INT8, wk::quantize_int8_weights)
  uint16_t* d_bf16;      // bf16 conv fragments (WK_PREC_BF16; BF16X3: hi then lo, wk::pack_fragments_bf16)
  int64_t ws_clips;
  int unfused;           // WAKEWORD_UNFUSED=1: front-end + CNN as two kernels (A/B testing)
  int fused_exp;         // WAKEWORD_FUSED_EXP, -DWK_DIAG builds only: role-isolation timing
                         // experiments (wrong logits); always 0 in the shipped library
  int fe_wg_per_cu = 2;  // standalone front-end workgroups per CU (WAKEWORD_FE_WG_PER_CU, -DWK_DIAG builds
                         // only: the occupancy experiment of DESIGN 5.1); 2 in the shipped library
};

namespace wk {

thread_local std::string g_last_error;

wk_status hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return WK_ERR_HIP;
}

wk_status invalid(const char* what) {
  g_last_error = what;
  return WK_ERR_INVALID_ARG;
}

wk_status fail(wk_status s, const char* what) {
  g_last_error = what;
  return s;
}

}  // namespace wk

using wk::g_last_error;
using wk::hip_fail;
using wk::invalid;
using wk::on_device;

namespace {

constexpr int64_t kWorkspaceClips = 16384;

}  // namespace

extern "C" {

int32_t wk_abi_version(void) { return WK_ABI_VERSION; }

const char* wk_status_string(wk_status s) {
  switch (s) {
    case WK_OK: return "WK_OK";
    case WK_ERR_INVALID_ARG: return "WK_ERR_INVALID_ARG";
    case WK_ERR_HIP: return "WK_ERR_HIP";
    case WK_ERR_NO_MEMORY: return "WK_ERR_NO_MEMORY";
    case WK_ERR_UNSUPPORTED: return "WK_ERR_UNSUPPORTED";
    case WK_ERR_DEVICE: return "WK_ERR_DEVICE";
  }
  return "WK_ERR_UNKNOWN";
}

const char* wk_last_error(void) { return g_last_error.c_str(); }

wk_status wk_create(const wk_config* cfg, const float* host_weights, wk_handle** out) {
  if (!cfg || !out) return invalid("wk_create: null cfg/out");
  *out = nullptr;
  if (cfg->mode != WK_MODE_TORCHAUDIO_CMVN && cfg->mode != WK_MODE_ESP_MFCC) return invalid("wk_create: bad mode");
  if (cfg->precision != WK_PREC_FP32 && cfg->precision != WK_PREC_BF16 && cfg->precision != WK_PREC_INT8 &&
      cfg->precision != WK_PREC_BF16X3)
    return invalid("wk_create: bad precision");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  if (cfg->device < 0 || cfg->device >= ndev) return invalid("wk_create: device ordinal out of range");
  wk_handle* h = new (std::nothrow) wk_handle();
  if (!h) return WK_ERR_NO_MEMORY;
  h->cfg = *cfg;
  {
    const char* u = getenv("WAKEWORD_UNFUSED");
    h->unfused = u && u[0] == '1';
#ifdef WK_DIAG
    const char* fx = getenv("WAKEWORD_FUSED_EXP");
    h->fused_exp = fx ? atoi(fx) : 0;
    const char* fw = getenv("WAKEWORD_FE_WG_PER_CU");
    if (fw && (atoi(fw) == 1 || atoi(fw) == 2)) h->fe_wg_per_cu = atoi(fw);
#endif
  }
  wk_status st = on_device(cfg->device, [&]() -> wk_status {
    hipDeviceProp_t prop;
    hipError_t e2 = hipGetDeviceProperties(&prop, cfg->device);
    if (e2 != hipSuccess) return hip_fail(e2, "hipGetDeviceProperties");
    h->n_cu = prop.multiProcessorCount;
    if ((e2 = hipHostMalloc(&h->h_err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
      return hip_fail(e2, "hipHostMalloc(error word)");
    *h->h_err = 0;
    if ((e2 = hipHostGetDevicePointer((void**)&h->d_err, h->h_err, 0)) != hipSuccess)
      return hip_fail(e2, "hipHostGetDevicePointer(error word)");
    if ((e2 = hipEventCreateWithFlags(&h->ws_free, hipEventDisableTiming)) != hipSuccess)
      return hip_fail(e2, "hipEventCreate");
    if (host_weights) {
      if ((e2 = hipMalloc(&h->d_weights, sizeof(float) * WK_NUM_WEIGHTS)) != hipSuccess)
        return hip_fail(e2, "hipMalloc(weights)");
      if ((e2 = hipMemcpy(h->d_weights, host_weights, sizeof(float) * WK_NUM_WEIGHTS, hipMemcpyHostToDevice)) !=
          hipSuccess)
        return hip_fail(e2, "hipMemcpy(weights)");
      std::vector<float> pk(wk::kNumPacked);
      wk::pack_fragments(host_weights, pk.data());
      if ((e2 = hipMalloc(&h->d_packed, sizeof(float) * wk::kNumPacked)) != hipSuccess)
        return hip_fail(e2, "hipMalloc(packed weights)");
      if ((e2 = hipMemcpy(h->d_packed, pk.data(), sizeof(float) * wk::kNumPacked, hipMemcpyHostToDevice)) !=
          hipSuccess)
        return hip_fail(e2, "hipMemcpy(packed weights)");
      if (cfg->precision == WK_PREC_BF16 || cfg->precision == WK_PREC_BF16X3) {
        const bool split = cfg->precision == WK_PREC_BF16X3;   // hi fragments, then lo fragments
        std::vector<uint16_t> pb(wk::kNumPackedBf16 * (split ? 2 : 1));
        wk::pack_fragments_bf16(host_weights, pb.data());
        if (split) wk::pack_fragments_bf16(host_weights, pb.data() + wk::kNumPackedBf16, true);
        if ((e2 = hipMalloc(&h->d_bf16, pb.size() * 2)) != hipSuccess) return hip_fail(e2, "hipMalloc(bf16 weights)");
        if ((e2 = hipMemcpy(h->d_bf16, pb.data(), pb.size() * 2, hipMemcpyHostToDevice)) != hipSuccess)
          return hip_fail(e2, "hipMemcpy(bf16 weights)");
      }
      if (cfg->precision == WK_PREC_INT8) {
        std::vector<int8_t> q(wk::kNumInt8Weights);
        wk::quantize_int8_weights(host_weights, q.data());
        if ((e2 = hipMalloc(&h->d_int8, q.size())) != hipSuccess) return hip_fail(e2, "hipMalloc(int8 weights)");
        if ((e2 = hipMemcpy(h->d_int8, q.data(), q.size(), hipMemcpyHostToDevice)) != hipSuccess)
          return hip_fail(e2, "hipMemcpy(int8 weights)");
      }
      h->ws_clips = kWorkspaceClips;
      if ((e2 = hipMalloc(&h->d_feats_ws, sizeof(float) * 13 * 63 * h->ws_clips)) != hipSuccess)
        return hip_fail(e2, "hipMalloc(workspace)");
    }
    return WK_OK;
  });
  if (st != WK_OK) {
    wk_destroy(h);
    return st;
  }
  *out = h;
  return WK_OK;
}

wk_status wk_destroy(wk_handle* h) {
  if (!h) return WK_OK;
  on_device(h->cfg.device, [&]() -> wk_status {
    if (h->d_weights) (void)hipFree(h->d_weights);
    if (h->d_feats_ws) (void)hipFree(h->d_feats_ws);
    if (h->d_packed) (void)hipFree(h->d_packed);
    if (h->d_int8) (void)hipFree(h->d_int8);
    if (h->d_bf16) (void)hipFree(h->d_bf16);
    if (h->ws_free) {
      (void)hipEventSynchronize(h->ws_free);
      (void)hipEventDestroy(h->ws_free);
    }
    if (h->h_err) (void)hipHostFree(h->h_err);
    return WK_OK;
  });
  delete h;
  return WK_OK;
}

wk_status wk_check_device_errors(wk_handle* h, uint32_t* flags_out) {
  if (!h) return invalid("wk_check_device_errors: null handle");
  return on_device(h->cfg.device, [&]() -> wk_status {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail(e, "wk_check_device_errors: sync");
    const uint32_t f = __atomic_exchange_n(h->h_err, 0u, __ATOMIC_SEQ_CST);
    if (flags_out) *flags_out = f;
    if (f) {
      g_last_error = "fused kernel protocol error (flags " + std::to_string(f) + "): logits since the last check are invalid";
      return WK_ERR_DEVICE;
    }
    return WK_OK;
  });
}

// Convolution arithmetic of the fused kernels (wk_fused.hip kConvF32 / kConvBf16 / kConvBf16x3).
static int conv_mode_of(const wk_handle* h) {
  return h->cfg.precision == WK_PREC_BF16 ? 1 : (h->cfg.precision == WK_PREC_BF16X3 ? 2 : 0);
}

static wk_status check_audio(const void* d_audio, int32_t dtype, int64_t batch, int32_t win_len, int64_t clip_stride,
                             bool mode_b) {
  if (batch < 0) return invalid("batch < 0");
  if (batch > 0 && !d_audio) return invalid("null audio pointer");
  if (dtype != WK_DTYPE_F32 && dtype != WK_DTYPE_I16) return invalid("bad dtype");
  if (mode_b && win_len != WK_WIN_SAMPLES) return invalid("mode B (torchaudio+CMVN) requires win_len == 16000");
  if (!mode_b && win_len < 320) return invalid("mode A requires win_len >= 320");
  if (batch > 1 && clip_stride < 1) return invalid("clip_stride < 1");   // < win_len = overlapping (sliding) windows
  return WK_OK;
}

wk_status wk_mfcc(wk_handle* h, const void* d_audio, int32_t dtype, int64_t batch, int32_t win_len,
                  int64_t clip_stride, float* d_feats, void* stream) {
  if (!h) return invalid("wk_mfcc: null handle");
  const bool mode_b = h->cfg.mode == WK_MODE_TORCHAUDIO_CMVN;
  wk_status s = check_audio(d_audio, dtype, batch, win_len, clip_stride, mode_b);
  if (s != WK_OK) return s;
  if (batch > 0 && !d_feats) return invalid("wk_mfcc: null feats");
  return on_device(h->cfg.device, [&]() -> wk_status {
    hipError_t e = wk::launch_frontend(mode_b, dtype == WK_DTYPE_I16, d_audio, batch, win_len, clip_stride, d_feats,
                                       h->cfg.esp_dsp_packing, h->cfg.cmvn, h->fe_wg_per_cu * h->n_cu, 0.97f,
                                       (hipStream_t)stream);
    return e == hipSuccess ? WK_OK : hip_fail(e, "frontend launch");
  });
}

wk_status wk_cnn(wk_handle* h, const float* d_feats, int64_t batch, float* d_logits, void* stream) {
  if (!h) return invalid("wk_cnn: null handle");
  if (!h->d_weights) return invalid("wk_cnn: handle created without weights");
  if (batch < 0 || (batch > 0 && (!d_feats || !d_logits))) return invalid("wk_cnn: bad arguments");
  return on_device(h->cfg.device, [&]() -> wk_status {
    hipError_t e = h->cfg.precision == WK_PREC_INT8
                       ? wk::launch_int8_cnn(d_feats, batch, h->d_int8, d_logits, 4 * h->n_cu, (hipStream_t)stream)
                       : wk::launch_cnn_fused(d_feats, batch, h->d_packed, h->d_bf16, conv_mode_of(h), d_logits, h->n_cu,
                                              (hipStream_t)stream, h->d_err);
    return e == hipSuccess ? WK_OK : hip_fail(e, "cnn launch");
  });
}

// wk_forward with the error word the launches report to: the handle's
// (wk_forward) or a stream object's own (wk_stream_push).
static wk_status forward_impl(wk_handle* h, const void* d_audio, int32_t dtype, int64_t batch, int32_t win_len,
                              int64_t clip_stride, float* d_logits, float* d_feats_or_null, void* stream,
                              unsigned* d_err) {
  if (!h) return invalid("wk_forward: null handle");
  if (h->cfg.mode != WK_MODE_TORCHAUDIO_CMVN) {
    g_last_error = "wk_forward: the xiaoa CNN consumes mode-B (torchaudio+CMVN) features";
    return WK_ERR_UNSUPPORTED;
  }
  if (!h->d_weights) return invalid("wk_forward: handle created without weights");
  wk_status s = check_audio(d_audio, dtype, batch, win_len, clip_stride, true);
  if (s != WK_OK) return s;
  if (batch > 0 && !d_logits) return invalid("wk_forward: null logits");
  const bool int8 = h->cfg.precision == WK_PREC_INT8;
  return on_device(h->cfg.device, [&]() -> wk_status {
    if (!h->unfused && !int8) {
      hipError_t e = wk::launch_fused(dtype == WK_DTYPE_I16, d_audio, batch, clip_stride, h->d_packed, h->d_bf16,
                                      conv_mode_of(h), d_logits, d_feats_or_null, h->n_cu, (hipStream_t)stream, d_err,
                                      h->fused_exp);
      return e == hipSuccess ? WK_OK : hip_fail(e, "fused launch");
    }
    const size_t esz = dtype == WK_DTYPE_I16 ? 2 : 4;
    // Features staged in the shared workspace: order this use after the last
    // one, whatever stream it ran on (a caller-provided feature buffer needs no ordering).
    std::unique_lock<std::mutex> ws_lock(h->ws_mu, std::defer_lock);
    if (!d_feats_or_null && batch > 0) {
      ws_lock.lock();
      if (h->ws_poisoned)
        return wk::fail(WK_ERR_HIP, "wk_forward: the feature workspace's previous use could not be ordered or drained");
      hipError_t e = h->ws_used ? hipStreamWaitEvent((hipStream_t)stream, h->ws_free, 0) : hipSuccess;
      if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent(workspace)");
    }
    // Every exit after the first launch (a failed later launch included) marks
    // the workspace busy until this stream's queued chunks are done, so the next
    // call on another stream still waits for them.  If the event cannot be
    // recorded, this stream is drained instead (the workspace is then idle)
    // and the failure is reported.
    bool launched = false;
    struct WsRelease {
      wk_handle* h;
      std::unique_lock<std::mutex>& lk;
      bool& launched;
      hipStream_t st;
      hipError_t release() {
        if (!lk.owns_lock() || !launched) return hipSuccess;
        launched = false;
        hipError_t e = hipEventRecord(h->ws_free, st);
        if (e == hipSuccess) {
          h->ws_used = true;
          return e;
        }
        if (hipStreamSynchronize(st) == hipSuccess || hipDeviceSynchronize() == hipSuccess) {
          h->ws_used = false;   // drained: nothing left to wait for
        } else {
          h->ws_poisoned = true;   // this call's chunks may still be queued: no later call may reuse the workspace
        }
        return e;
      }
      ~WsRelease() { (void)release(); }
    } ws_release{h, ws_lock, launched, (hipStream_t)stream};
    for (int64_t c0 = 0; c0 < batch; c0 += h->ws_clips) {
      const int64_t n = batch - c0 < h->ws_clips ? batch - c0 : h->ws_clips;
      float* feats = d_feats_or_null ? d_feats_or_null + c0 * 13 * 63 : h->d_feats_ws;
      const void* a = (const char*)d_audio + (size_t)(c0 * clip_stride) * esz;
      launched = true;   // (a failed launch may still have queued work)
      hipError_t e = wk::launch_frontend(true, dtype == WK_DTYPE_I16, a, n, win_len, clip_stride, feats, 0, 1,
                                         2 * h->n_cu, 0.97f, (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(e, "frontend launch");
      e = int8 ? wk::launch_int8_cnn(feats, n, h->d_int8, d_logits + c0, 4 * h->n_cu, (hipStream_t)stream)
               : wk::launch_cnn_fused(feats, n, h->d_packed, h->d_bf16, conv_mode_of(h), d_logits + c0, h->n_cu,
                                      (hipStream_t)stream, d_err);
      if (e != hipSuccess) return hip_fail(e, "cnn launch");
    }
    const hipError_t er = ws_release.release();
    if (er != hipSuccess) return hip_fail(er, "hipEventRecord(workspace)");
    return WK_OK;
  });
}

wk_status wk_forward(wk_handle* h, const void* d_audio, int32_t dtype, int64_t batch, int32_t win_len,
                     int64_t clip_stride, float* d_logits, float* d_feats_or_null, void* stream) {
  return forward_impl(h, d_audio, dtype, batch, win_len, clip_stride, d_logits, d_feats_or_null, stream,
                      h ? h->d_err : nullptr);
}

wk_status wk_synth_clips(uint32_t seed, int64_t first, int64_t count, int32_t n, float* d_out, void* stream) {
  if (count < 0 || n <= 0 || (count > 0 && !d_out)) return invalid("wk_synth_clips: bad arguments");
  hipError_t e = wk::launch_synth(seed, first, count, n, d_out, (hipStream_t)stream);
  return e == hipSuccess ? WK_OK : hip_fail(e, "synth launch");
}

wk_status wk_normalize(const float* d_in, float* d_out, int64_t batch, int32_t n_coef, int32_t n_time,
                       int32_t method, void* stream) {
  if (batch < 0 || n_coef <= 0 || n_time <= 1 || method < 0 || method > 3) return invalid("wk_normalize: bad args");
  if (batch > 0 && (!d_in || !d_out)) return invalid("wk_normalize: null pointer");
  hipError_t e = wk::launch_normalize(d_in, d_out, batch, n_coef, n_time, method, (hipStream_t)stream);
  return e == hipSuccess ? WK_OK : hip_fail(e, "normalize launch");
}

wk_status wk_record_front(const int16_t* d_tdm, int64_t n_out, int16_t* d_out16, float* d_out_f32_or_null,
                          void* stream) {
  if (n_out < 0 || (n_out > 0 && (!d_tdm || !d_out16))) return invalid("wk_record_front: bad arguments");
  if (n_out > 1 && ((uintptr_t)d_tdm & 15)) return invalid("wk_record_front: d_tdm must be 16-byte aligned");
  if (((uintptr_t)d_out16 & 3) || ((uintptr_t)d_out_f32_or_null & 7))
    return invalid("wk_record_front: d_out16 must be 4-byte and d_out_f32 8-byte aligned");
  hipError_t e = wk::launch_record_front(d_tdm, n_out, d_out16, d_out_f32_or_null, (hipStream_t)stream);
  return e == hipSuccess ? WK_OK : hip_fail(e, "record_front launch");
}

wk_status wk_quantize_frames(const float* d_mfcc, int64_t n_values, int8_t* d_out_i8, void* stream) {
  if (n_values < 0 || (n_values > 0 && (!d_mfcc || !d_out_i8))) return invalid("wk_quantize_frames: bad arguments");
  hipError_t e = wk::launch_quantize_frames(d_mfcc, n_values, d_out_i8, (hipStream_t)stream);
  return e == hipSuccess ? WK_OK : hip_fail(e, "quantize_frames launch");
}

wk_status wk_device_cmvn(const void* d_frames, int32_t dtype, int64_t n_frames, int8_t* d_out_i8,
                         float* d_feats_or_null, void* stream) {
  if (n_frames < 0 || (dtype != WK_DTYPE_I8 && dtype != WK_DTYPE_F32)) return invalid("wk_device_cmvn: bad args");
  if (!d_out_i8 && !d_feats_or_null) return invalid("wk_device_cmvn: no output");
  const int64_t n_windows = n_frames >= 63 ? n_frames - 62 : 0;
  if (n_windows > 0 && !d_frames) return invalid("wk_device_cmvn: null frames");
  hipError_t e = wk::launch_device_cmvn(d_frames, dtype == WK_DTYPE_I8, n_windows, d_out_i8, d_feats_or_null,
                                        (hipStream_t)stream);
  return e == hipSuccess ? WK_OK : hip_fail(e, "device_cmvn launch");
}

// ---------------------------------------------------------------------------
// mfcc.h compatibility shims (main/esp_mfcc/mfcc.h:10-17, mfcc.c:431-563).
// ---------------------------------------------------------------------------
}  // extern "C"

static std::mutex g_compat_mu;
static wk_handle* g_compat = nullptr;

// The fixed-geometry mode-A handle of the shims (reference configuration).
static bool compat_handle() {
  if (g_compat) return true;
  wk_config cfg = {WK_MODE_ESP_MFCC, WK_PREC_FP32, 1, 0, 0};
  if (wk_create(&cfg, nullptr, &g_compat) != WK_OK) {
    fprintf(stderr, "E (MFCC) device init failed: %s\n", wk_last_error());
    return false;
  }
  return true;
}

// Every other parameter set: wk_esp_mfcc objects, cached per parameter set
// (mfcc.c rebuilds its tables per call; the single-frame variant caches its
// filterbank per (sr, n_filters, n_fft), mfcc.c:362-377).  Caller holds g_compat_mu.
struct EspKey {
  int sr, frame, n_fft, n_filters, n_mfcc;
  bool operator==(const EspKey& o) const {
    return sr == o.sr && frame == o.frame && n_fft == o.n_fft && n_filters == o.n_filters && n_mfcc == o.n_mfcc;
  }
};
static std::vector<std::pair<EspKey, wk_esp_mfcc*>> g_esp_cache;
static wk_esp_mfcc* esp_object(const EspKey& k) {
  for (auto& e : g_esp_cache)
    if (e.first == k) return e.second;
  wk_esp_mfcc* m = nullptr;
  if (wk_esp_mfcc_create(k.sr, k.frame, k.n_fft, k.n_filters, k.n_mfcc, 1, 0, &m) != WK_OK) return nullptr;
  if (g_esp_cache.size() >= 8) {   // oldest out
    (void)wk_esp_mfcc_destroy(g_esp_cache.front().second);
    g_esp_cache.erase(g_esp_cache.begin());
  }
  g_esp_cache.emplace_back(k, m);
  return m;
}

// Host signal -> malloc'd host [nf][n_mfcc] through the device: `run` fills
// d_out from d_sig.  Caller holds g_compat_mu.
template <class F>
static float* shim_run(const float* signal, int n_in, size_t n_out, const char* what, F run) {
  float* host_out = (float*)malloc(sizeof(float) * (n_out ? n_out : 1));
  if (!host_out) return nullptr;
  float *d_sig = nullptr, *d_out = nullptr;
  const wk_status st = on_device(0, [&]() -> wk_status {
    hipError_t e;
    if ((e = hipMalloc(&d_sig, sizeof(float) * n_in)) != hipSuccess) return hip_fail(e, "hipMalloc");
    if ((e = hipMalloc(&d_out, sizeof(float) * (n_out ? n_out : 1))) != hipSuccess) return hip_fail(e, "hipMalloc");
    if ((e = hipMemcpy(d_sig, signal, sizeof(float) * n_in, hipMemcpyHostToDevice)) != hipSuccess)
      return hip_fail(e, "H2D");
    const wk_status s = run(d_sig, d_out);
    if (s != WK_OK) return s;
    if ((e = hipMemcpy(host_out, d_out, sizeof(float) * n_out, hipMemcpyDeviceToHost)) != hipSuccess)
      return hip_fail(e, "D2H");
    return WK_OK;
  });
  on_device(0, [&]() -> wk_status {
    if (d_sig) (void)hipFree(d_sig);
    if (d_out) (void)hipFree(d_out);
    return WK_OK;
  });
  if (st != WK_OK) {
    fprintf(stderr, "E (MFCC) %s failed: %s\n", what, wk_last_error());
    free(host_out);
    return nullptr;
  }
  return host_out;
}

extern "C" {

float* extract_mfcc(const float* signal, int signal_len, int sampling_rate, int frame_size, int hop_size, int n_fft,
                    int n_filters, int n_mfcc) {
  // mfcc.c:434-437: NULL signal or a signal shorter than one frame -> NULL.
  if (!signal || signal_len < frame_size || frame_size <= 0) {
    fprintf(stderr, "E (MFCC) Invalid signal parameters\n");
    return nullptr;
  }
  if (hop_size < 1) {   // (mfcc.c:447 divides by it)
    fprintf(stderr, "E (MFCC) Invalid hop size\n");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_compat_mu);
  const int nf = (signal_len - frame_size) / hop_size + 1;
  const size_t n_out = (size_t)nf * n_mfcc;
  if (sampling_rate == 16000 && frame_size == 320 && hop_size == 256 && n_fft == 512 && n_filters == 40 &&
      n_mfcc == 13) {
    if (!compat_handle()) return nullptr;
    return shim_run(signal, signal_len, n_out, "extract_mfcc", [&](float* d_sig, float* d_out) {
      return wk_mfcc(g_compat, d_sig, WK_DTYPE_F32, 1, signal_len, signal_len, d_out, nullptr);
    });
  }
  wk_esp_mfcc* m = esp_object({sampling_rate, frame_size, n_fft, n_filters, n_mfcc});
  if (!m) {
    fprintf(stderr, "E (MFCC) unsupported configuration: %s\n", wk_last_error());
    return nullptr;
  }
  return shim_run(signal, signal_len, n_out, "extract_mfcc", [&](float* d_sig, float* d_out) {
    return wk_esp_mfcc_run(m, d_sig, 1, signal_len, signal_len, hop_size, 0.97f, d_out, nullptr);
  });
}

void free_mfcc(float* mfcc) { free(mfcc); }

// mfcc.c:297-427 flow_extract_mfcc_single_frame: one frame, NO pre-emphasis,
// symmetric Hamming over frame_size, |FFT|^2/n_fft + 1e-12 (esp-dsp packing),
// mel, ln, DCT-II -> malloc'd n_mfcc floats (free with free_mfcc), NULL on bad
// arguments (mfcc.c:300-303).  The reference configuration (320-sample frame,
// 16 kHz, 512, 40 filters, n_mfcc <= 13) runs on the fixed-geometry kernel,
// any other on wk_esp_mfcc.
float* flow_extract_mfcc_single_frame(const float* frame, int frame_size, int sampling_rate, int n_fft, int n_filters,
                                      int n_mfcc) {
  if (!frame || frame_size <= 0 || frame_size > n_fft) {
    fprintf(stderr, "E (MFCC) Invalid frame parameters\n");
    return nullptr;
  }
  if (n_mfcc < 1) {
    fprintf(stderr, "E (MFCC) Invalid n_mfcc\n");
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_compat_mu);
  if (sampling_rate == 16000 && frame_size == 320 && n_fft == 512 && n_filters == 40 && n_mfcc <= 13) {
    if (!compat_handle()) return nullptr;
    float* all = shim_run(frame, frame_size, 13, "flow_extract_mfcc_single_frame", [&](float* d_sig, float* d_out) {
      const hipError_t e = wk::launch_frontend(false, false, d_sig, 1, frame_size, frame_size, d_out, 1, 0, 1, 0.0f,
                                               nullptr);
      return e == hipSuccess ? WK_OK : hip_fail(e, "frontend launch");
    });
    return all;   // (the first n_mfcc of the 13 are the caller's; the block is larger than it needs)
  }
  wk_esp_mfcc* m = esp_object({sampling_rate, frame_size, n_fft, n_filters, n_mfcc});
  if (!m) {
    fprintf(stderr, "E (MFCC) unsupported configuration: %s\n", wk_last_error());
    return nullptr;
  }
  return shim_run(frame, frame_size, (size_t)n_mfcc, "flow_extract_mfcc_single_frame", [&](float* d_sig, float* d_out) {
    return wk_esp_mfcc_run(m, d_sig, 1, frame_size, frame_size, frame_size, 0.0f, d_out, nullptr);
  });
}

// mfcc.c:530-553: min/max/avg over the finite entries.
void analyze_mfcc_range(float* mfcc, int size, const char* label) {
  if (!mfcc || size <= 0) return;
  float mn = INFINITY, mx = -INFINITY, sum = 0.0f;
  int valid = 0;
  for (int i = 0; i < size; i++) {
    if (!isnan(mfcc[i]) && !isinf(mfcc[i])) {
      if (mfcc[i] < mn) mn = mfcc[i];
      if (mfcc[i] > mx) mx = mfcc[i];
      sum += mfcc[i];
      valid++;
    }
  }
  if (valid > 0)
    printf("I (MFCC) %s MFCC Range: min=%.6f, max=%.6f, avg=%.6f, valid=%d/%d\n", label ? label : "", mn, mx,
           sum / valid, valid, size);
  else
    fprintf(stderr, "E (MFCC) %s MFCC: No valid values\n", label ? label : "");
  fflush(stdout);
}

// ---------------------------------------------------------------------------
// Streaming ring.
//
// A ring of `cap` float samples, stored mirrored (sample p at p % cap and
// p % cap + cap), so every window of <= cap samples is contiguous and a run of
// consecutive windows is one strided wk_forward launch.  Writes follow
// ring_buffer.c:57-117 (write_rinbuffer): a push longer than the ring keeps
// only its newest `cap` samples, older data is overwritten.  Window k covers
// stream samples [k*hop, k*hop + 16000); a push completes every window whose
// end it reaches; windows whose start was already overwritten are dropped.
//
// The mirrored ring is in device memory.  A push writes its samples once into
// a pinned, mapped host staging ring of `cap` (same positions); a push that
// completes windows first launches wk_ring_ingest_kernel, which reads the
// samples pushed since the last launch (only the newest `cap`: older ones are
// overwritten, and no window left to score starts there) across PCIe into both
// copies of the device ring, then the fused kernel reads its windows from HBM
// and writes the logits straight into pinned host memory -- two launches and
// one wait per push, no copy commands.  (Reading each window across PCIe
// instead, zero-copy from a mirrored host ring, cost ~9 us per window: one
// workgroup's loads over PCIe latency; a hop of new samples is one round trip.)
// ---------------------------------------------------------------------------

struct wk_stream {
  wk_handle* h;
  hipStream_t st;
  int32_t hop, cap;
  int64_t total;        // samples pushed since create / reset
  int64_t next_win;     // index of the next window to score
  int64_t ingested;     // stream samples [0, ingested) are in d_ring (as far as it holds them)
  float* h_ring;        // pinned, mapped [cap] staging ring (written by the host, read by the ingest kernel)
  float* a_ring;        // device alias of h_ring
  float* d_ring;        // device [2*cap], mirrored: sample p at p % cap and p % cap + cap
  float* h_logits;      // pinned, mapped [max_win] (written by the kernel)
  float* a_logits;      // device alias of h_logits
  unsigned* h_err;      // pinned, mapped: this stream object's own error word (its pushes' launches only)
  unsigned* d_err;      // device alias of h_err
  int32_t max_win;
};

static void stream_free(wk_stream* s) {
  (void)hipHostFree(s->h_ring);
  (void)hipFree(s->d_ring);
  (void)hipHostFree(s->h_logits);
  (void)hipHostFree(s->h_err);
  free(s);
}

wk_status wk_stream_create(wk_handle* h, int32_t hop, int32_t capacity, void* stream, wk_stream** out) {
  if (!h || !out) return invalid("wk_stream_create: null argument");
  if (hop < 1 || capacity < WK_WIN_SAMPLES + hop) return invalid("wk_stream_create: need hop >= 1, capacity >= 16000 + hop");
  if (h->cfg.mode != WK_MODE_TORCHAUDIO_CMVN || !h->d_weights)
    return invalid("wk_stream_create: needs a mode-B handle with weights");
  *out = nullptr;
  return on_device(h->cfg.device, [&]() -> wk_status {
    wk_stream* s = (wk_stream*)calloc(1, sizeof(wk_stream));
    if (!s) return WK_ERR_NO_MEMORY;
    s->h = h;
    s->st = (hipStream_t)stream;
    s->hop = hop;
    s->cap = capacity;
    s->max_win = (capacity - WK_WIN_SAMPLES) / hop + 1;
    const unsigned mapped = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e;
    if ((e = hipHostMalloc(&s->h_ring, sizeof(float) * (size_t)capacity, mapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&s->a_ring, s->h_ring, 0)) != hipSuccess ||
        (e = hipMalloc(&s->d_ring, sizeof(float) * 2 * (size_t)capacity)) != hipSuccess ||
        (e = hipHostMalloc(&s->h_logits, sizeof(float) * (size_t)s->max_win, mapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&s->a_logits, s->h_logits, 0)) != hipSuccess ||
        (e = hipHostMalloc(&s->h_err, sizeof(unsigned), mapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&s->d_err, s->h_err, 0)) != hipSuccess) {
      stream_free(s);
      return e == hipErrorOutOfMemory ? WK_ERR_NO_MEMORY : hip_fail(e, "wk_stream_create");
    }
    memset(s->h_ring, 0, sizeof(float) * (size_t)capacity);
    *s->h_err = 0;
    *out = s;
    return WK_OK;
  });
}

wk_status wk_stream_destroy(wk_stream* s) {
  if (!s) return WK_OK;
  return on_device(s->h->cfg.device, [&]() -> wk_status {
    (void)hipStreamSynchronize(s->st);
    stream_free(s);
    return WK_OK;
  });
}

wk_status wk_stream_reset(wk_stream* s) {
  if (!s) return invalid("wk_stream_reset: null stream");
  s->total = 0;
  s->next_win = 0;
  s->ingested = 0;
  return WK_OK;
}

wk_status wk_stream_push(wk_stream* s, const float* samples, int64_t n, float* out_logits, int64_t* out_end,
                         int32_t max_out, int32_t* n_out) {
  if (!s || !n_out || n < 0 || (n > 0 && !samples) || max_out < 0 || (max_out > 0 && !out_logits))
    return invalid("wk_stream_push: bad arguments");
  *n_out = 0;
  // Every push that launches work waits for it before returning, so no kernel
  // is reading the host staging ring while it is rewritten here.
  const int64_t cap = s->cap;
  // 1. ring write (overwrite-oldest): only the newest `cap` samples of a long push survive.
  const int64_t skip = n > cap ? n - cap : 0;
  const int64_t m = n - skip;
  const int64_t p0 = s->total + skip;
  for (int64_t done = 0; done < m;) {   // at most two segments (wrap)
    const int64_t pos = (p0 + done) % cap;
    const int64_t len = m - done < cap - pos ? m - done : cap - pos;
    memcpy(s->h_ring + pos, samples + skip + done, sizeof(float) * (size_t)len);
    done += len;
  }
  s->total += n;
  // 2. windows completed by this push whose start is still in the ring.
  const int64_t last = s->total >= WK_WIN_SAMPLES ? (s->total - WK_WIN_SAMPLES) / s->hop : -1;
  int64_t first = s->next_win;
  const int64_t oldest = s->total > cap ? (s->total - cap + s->hop - 1) / s->hop : 0;
  if (first < oldest) first = oldest;
  if (last - first + 1 > max_out) first = last - max_out + 1;   // report the newest max_out
  s->next_win = last + 1 > s->next_win ? last + 1 : s->next_win;
  const int64_t k = last - first + 1;
  if (k <= 0) return WK_OK;
  return on_device(s->h->cfg.device, [&]() -> wk_status {
    // 3. score them: contiguous strided runs in the mirrored ring.  On any
    // failure after the first launch the stream is drained before returning,
    // so no kernel is still reading the host ring when the next push rewrites it.
    struct Drain {
      hipStream_t st;
      bool armed = false;
      ~Drain() {
        if (armed) (void)hipStreamSynchronize(st);
      }
    } drain{s->st};
    hipError_t e;
    // the samples pushed since the last launch that the staging ring still holds
    const int64_t from = s->ingested > s->total - cap ? s->ingested : s->total - cap;
    drain.armed = true;
    if ((e = wk::launch_ring_ingest(s->a_ring, s->d_ring, cap, from % cap, s->total - from, s->st)) != hipSuccess)
      return hip_fail(e, "wk_stream_push: ingest");
    s->ingested = s->total;
    int64_t w = first;
    while (w <= last) {
      const int64_t off = (w * s->hop) % cap;
      int64_t run = (2 * cap - WK_WIN_SAMPLES - off) / s->hop + 1;   // windows that fit before the mirror end
      if (run > last - w + 1) run = last - w + 1;
      wk_status st = forward_impl(s->h, s->d_ring + off, WK_DTYPE_F32, run, WK_WIN_SAMPLES, s->hop,
                                  s->a_logits + (w - first), nullptr, s->st, s->d_err);
      if (st != WK_OK) return st;
      w += run;
    }
    if ((e = hipStreamSynchronize(s->st)) != hipSuccess) return hip_fail(e, "wk_stream_push: sync");
    drain.armed = false;
    // synced, and only this stream object's launches report to its word: final
    if (const uint32_t f = __atomic_exchange_n(s->h_err, 0u, __ATOMIC_SEQ_CST)) {
      g_last_error = "fused kernel protocol error (flags " + std::to_string(f) + "): these logits are invalid";
      return WK_ERR_DEVICE;
    }
    memcpy(out_logits, s->h_logits, sizeof(float) * (size_t)k);
    if (out_end)
      for (int64_t i = 0; i < k; ++i) out_end[i] = (first + i) * s->hop + WK_WIN_SAMPLES;
    *n_out = (int32_t)k;
    return WK_OK;
  });
}

}  // extern "C"
