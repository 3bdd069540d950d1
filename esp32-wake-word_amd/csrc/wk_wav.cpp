// wk_wav.cpp -- host-side WAV ingest and waveform augmentation (SURVEY 8(f)
// item 4): the data formats on the input side of the hot path.  Pure host
// C++ (no device code), compiled into both libwakeword.so and
// libwakeword_host.so: it fills caller buffers -- typically pinned host
// memory handed to wk_forward's H2D copy, or the host path's input.
//
//   wk_wav_read        esp_wav.cpp:8-139  (RIFF / WAVE / "fmt " header, unknown
//                      chunks before "data" skipped, PCM16, truncation)
//   wk_wav_load_batch  torchaudio.load scaling (x / 32768) + pad_audio
//                      (extract_mfcc.py:7-23), many files on worker threads
//   wk_augment         augment_audio_waveform (extract_mfcc.py:90-121): speed
//                      change by linear interpolation (F.interpolate,
//                      align_corners=False) + pad/trim, volume x v + clamp
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "wakeword.h"
#include "wk_status.h"

using wk::fail;
using wk::invalid;

namespace {

struct FileCloser {
  FILE* f;
  ~FileCloser() {
    if (f) fclose(f);
  }
};

bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

// Parse the header; leaves the stream at the first data byte.
wk_status parse_header(FILE* f, wk_wav_info* info) {
  char tag[4];
  uint32_t riff_len, fmt_len, u32;
  uint16_t fmt, ch, bps, align;
  if (!rd(f, tag, 4) || memcmp(tag, "RIFF", 4) != 0) return invalid("wk_wav_read: not a RIFF file");
  if (!rd(f, &riff_len, 4) || !rd(f, tag, 4) || memcmp(tag, "WAVE", 4) != 0)
    return invalid("wk_wav_read: missing WAVE tag");
  // The reference expects "fmt " right after WAVE (esp_wav.cpp:55-66); other
  // chunks are skipped only while searching for "data" (:101-126).  Be as
  // lenient for chunks before "fmt " as for those before "data".
  for (;;) {
    if (!rd(f, tag, 4) || !rd(f, &fmt_len, 4)) return invalid("wk_wav_read: no fmt chunk");
    if (memcmp(tag, "fmt ", 4) == 0) break;
    if (fseek(f, (long)fmt_len + (fmt_len & 1), SEEK_CUR) != 0) return invalid("wk_wav_read: truncated chunk");
  }
  if (fmt_len < 16 || !rd(f, &fmt, 2) || !rd(f, &ch, 2) || !rd(f, &u32, 4)) return invalid("wk_wav_read: short fmt");
  info->sample_rate = (int32_t)u32;
  if (!rd(f, &u32, 4) || !rd(f, &align, 2) || !rd(f, &bps, 2)) return invalid("wk_wav_read: short fmt");
  if (fmt_len > 16 && fseek(f, (long)(fmt_len - 16) + (fmt_len & 1), SEEK_CUR) != 0)
    return invalid("wk_wav_read: short fmt");
  info->channels = ch;
  info->bits_per_sample = bps;
  if (fmt != 1 || bps != 16) return fail(WK_ERR_UNSUPPORTED, "wk_wav_read: only PCM 16-bit is supported");
  if (ch < 1) return invalid("wk_wav_read: zero channels");
  for (;;) {   // find "data", skipping unknown chunks (esp_wav.cpp:101-126)
    uint32_t sz;
    if (!rd(f, tag, 4) || !rd(f, &sz, 4)) return invalid("wk_wav_read: data chunk not found");
    if (memcmp(tag, "data", 4) == 0) {
      info->data_samples = (int32_t)(sz / (2u * ch));
      return WK_OK;
    }
    if (fseek(f, (long)sz + (sz & 1), SEEK_CUR) != 0) return invalid("wk_wav_read: truncated chunk");
  }
}

wk_status read_one(const char* path, int16_t* out, int32_t max_samples, wk_wav_info* info) {
  FileCloser fc{fopen(path, "rb")};
  if (!fc.f) return invalid("wk_wav_read: cannot open file");
  wk_status s = parse_header(fc.f, info);
  if (s != WK_OK) return s;
  // Channel 0 of interleaved frames (the reference files are mono).
  const int32_t n = std::min(info->data_samples, max_samples);
  const int ch = info->channels;
  if (ch == 1) {
    info->n_samples = (int32_t)fread(out, 2, (size_t)n, fc.f);
  } else {
    std::vector<int16_t> fr((size_t)ch);
    int32_t i = 0;
    for (; i < n && fread(fr.data(), 2, (size_t)ch, fc.f) == (size_t)ch; ++i) out[i] = fr[0];
    info->n_samples = i;
  }
  return WK_OK;
}

// Counter-hash N(0,1) (Box-Muller), keyed on (seed, stream, index).
uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
float gauss(uint32_t seed, uint32_t stream, uint32_t i) {
  const uint32_t k = mix32(seed ^ (stream * 0x9E3779B9u));
  const uint32_t h1 = mix32(k ^ (i * 2u + 0x68E31DA4u)), h2 = mix32(h1 ^ 0xB5297A4Du);
  const float u1 = ((float)(h1 >> 8) + 1.0f) * (1.0f / 16777216.0f), u2 = (float)(h2 >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.28318530717958648f * u2);
}

}  // namespace

extern "C" {

wk_status wk_wav_read(const char* path, int16_t* out, int32_t max_samples, wk_wav_info* info) {
  if (!path || !info || max_samples < 0 || (max_samples > 0 && !out)) return invalid("wk_wav_read: bad arguments");
  memset(info, 0, sizeof(*info));
  return read_one(path, out, max_samples, info);
}

wk_status wk_wav_load_batch(const char* const* paths, int32_t n, int32_t pad_to, float noise_level, uint32_t seed,
                            float* out, int32_t* n_read) {
  if (n < 0 || pad_to <= 0 || (n > 0 && (!paths || !out)) || noise_level < 0.0f)
    return invalid("wk_wav_load_batch: bad arguments");
  std::atomic<int32_t> next{0};
  std::atomic<int> first_err{WK_OK};
  std::string err;
  auto worker = [&]() {
    std::vector<int16_t> buf((size_t)pad_to);
    for (int32_t i; (i = next.fetch_add(1)) < n;) {
      wk_wav_info info;
      memset(&info, 0, sizeof(info));
      const wk_status s = read_one(paths[i], buf.data(), pad_to, &info);
      float* o = out + (size_t)i * pad_to;
      if (s != WK_OK) {
        int expect = WK_OK;
        if (first_err.compare_exchange_strong(expect, (int)s)) err = wk::g_last_error + " (" + paths[i] + ")";
        std::fill(o, o + pad_to, 0.0f);
        continue;
      }
      for (int32_t j = 0; j < info.n_samples; ++j) o[j] = (float)buf[j] * (1.0f / 32768.0f);   // torchaudio.load
      for (int32_t j = info.n_samples; j < pad_to; ++j)   // pad_audio: N(0, noise_level^2) or zeros
        o[j] = noise_level > 0.0f ? noise_level * gauss(seed, (uint32_t)i, (uint32_t)j) : 0.0f;
      if (n_read) n_read[i] = info.n_samples;
    }
  };
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const int nt = (int)std::min<int64_t>(hw, n);
  std::vector<std::thread> ts;
  for (int t = 1; t < nt; ++t) ts.emplace_back(worker);
  worker();
  for (auto& t : ts) t.join();
  if (first_err.load() != WK_OK) {
    wk::g_last_error = err;
    return (wk_status)first_err.load();
  }
  return WK_OK;
}

wk_status wk_augment(const float* in, int32_t n, float speed, float volume, float noise_level, uint32_t seed, float* out,
                     int32_t out_len) {
  if (!in || !out || n <= 0 || out_len <= 0 || !(speed > 0.0f) || !(volume > 0.0f) || noise_level < 0.0f)
    return invalid("wk_augment: bad arguments");
  // speed: F.interpolate(size=int(n * speed), mode='linear', align_corners=False), then pad/trim to out_len
  const double md = (double)n * (double)speed;   // (range-checked before the cast: UBSan, tests/test_sanitizers.py)
  if (!(md >= 1.0) || md > 2147483647.0) return invalid("wk_augment: speed out of range");
  const int32_t m = (int32_t)md;
  const float scale = (float)n / (float)m;
  for (int32_t i = 0; i < out_len; ++i) {
    float v = noise_level > 0.0f ? noise_level * gauss(seed, 0u, (uint32_t)i) : 0.0f;   // pad_audio's noise pad
    if (i < m) {
      float src = scale * ((float)i + 0.5f) - 0.5f;
      src = src < 0.0f ? 0.0f : src;
      const int32_t i0 = (int32_t)src;
      const int32_t i1 = i0 + (i0 < n - 1 ? 1 : 0);
      const float l1 = src - (float)i0, l0 = 1.0f - l1;
      v = l0 * in[i0] + l1 * in[i1];
    }
    v *= volume;   // volume change with clamp to [-1, 1]
    out[i] = volume != 1.0f ? std::min(1.0f, std::max(-1.0f, v)) : v;
  }
  return WK_OK;
}

}  // extern "C"
