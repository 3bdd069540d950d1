// Host-only ASan/UBSan harness for the WAV ingest (csrc/wk_wav.cpp, the
// replacement of esp_wav.cpp:8-139) -- test infrastructure, built and run by
// tests/test_sanitizers.py on the CPU (never on the GPU box).
//
//   wav_harness <scratch_dir> <wav> [<wav> ...]
//
// For every reference WAV: the file itself; every truncation of its first
// 128 bytes and a sample of longer ones; single-byte corruptions of every
// header byte (chunk sizes become huge, odd, zero); chunk ids swapped; an
// odd-sized unknown chunk before "fmt " and before "data"; a stereo and a
// 24-bit variant.  Each goes through wk_wav_read (small and large
// max_samples) and wk_wav_load_batch; wk_augment runs over edge arguments.
// Any sanitizer report aborts the process (-fno-sanitize-recover=all).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "wakeword.h"

namespace wk {   // the error helpers wk_api.hip defines for the product library
thread_local std::string g_last_error;
wk_status invalid(const char* what) {
  g_last_error = what;
  return WK_ERR_INVALID_ARG;
}
wk_status fail(wk_status s, const char* what) {
  g_last_error = what;
  return s;
}
}  // namespace wk

static std::vector<uint8_t> slurp(const char* p) {
  std::vector<uint8_t> v;
  FILE* f = fopen(p, "rb");
  if (!f) return v;
  uint8_t b[4096];
  size_t n;
  while ((n = fread(b, 1, sizeof b, f)) > 0) v.insert(v.end(), b, b + n);
  fclose(f);
  return v;
}

static void put(const std::string& p, const std::vector<uint8_t>& v) {
  FILE* f = fopen(p.c_str(), "wb");
  if (!f) abort();
  if (!v.empty() && fwrite(v.data(), 1, v.size(), f) != v.size()) abort();
  fclose(f);
}

static long g_cases = 0, g_ok = 0;

static void run_file(const std::string& p) {
  static std::vector<int16_t> buf(1 << 20);
  for (int32_t mx : {0, 1, 333, 16000, 1 << 20}) {
    wk_wav_info info;
    const wk_status s = wk_wav_read(p.c_str(), buf.data(), mx, &info);
    ++g_cases;
    if (s == WK_OK) {
      ++g_ok;
      if (info.n_samples < 0 || info.n_samples > mx) abort();
    }
  }
  std::vector<float> out(3 * 4000);
  int32_t nr[3] = {0, 0, 0};
  const char* paths[3] = {p.c_str(), p.c_str(), p.c_str()};
  (void)wk_wav_load_batch(paths, 3, 4000, 0.005f, 7u, out.data(), nr);
  for (int i = 0; i < 3; ++i)
    if (nr[i] < 0 || nr[i] > 4000) abort();
}

static void put_u32(std::vector<uint8_t>& v, size_t at, uint32_t x) { memcpy(v.data() + at, &x, 4); }

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string dir = argv[1];
  const std::string tmp = dir + "/case.wav";
  for (int a = 2; a < argc; ++a) {
    const std::vector<uint8_t> w = slurp(argv[a]);
    if (w.size() < 44) return 3;
    put(tmp, w);
    run_file(tmp);
    // truncations
    for (size_t n = 0; n < w.size(); n += (n < 128 ? 1 : 997)) {
      put(tmp, std::vector<uint8_t>(w.begin(), w.begin() + n));
      run_file(tmp);
    }
    // single-byte corruptions of the header
    for (size_t i = 0; i < 64 && i < w.size(); ++i)
      for (uint8_t x : {0x00, 0x01, 0x7F, 0x80, 0xFF}) {
        std::vector<uint8_t> c = w;
        c[i] = x;
        put(tmp, c);
        run_file(tmp);
      }
    // odd-sized unknown chunks before "fmt " and before "data"
    for (uint32_t odd : {1u, 3u, 7u, 0xFFFFFFF1u}) {
      std::vector<uint8_t> c(w.begin(), w.begin() + 12);
      const uint8_t junk[8] = {'J', 'U', 'N', 'K', 0, 0, 0, 0};
      c.insert(c.end(), junk, junk + 8);
      put_u32(c, 16, odd);
      c.insert(c.end(), odd < 64 ? odd + (odd & 1) : 0, 0x55);
      c.insert(c.end(), w.begin() + 12, w.end());
      put(tmp, c);
      run_file(tmp);
    }
    {   // "LIST" chunk between fmt and data, odd length
      std::vector<uint8_t> c(w.begin(), w.begin() + 36);
      const uint8_t list[8] = {'L', 'I', 'S', 'T', 5, 0, 0, 0};
      c.insert(c.end(), list, list + 8);
      c.insert(c.end(), 6, 0x41);
      c.insert(c.end(), w.begin() + 36, w.end());
      put(tmp, c);
      run_file(tmp);
    }
    {   // stereo, and 24-bit (unsupported) declared in the fmt chunk
      std::vector<uint8_t> c = w;
      c[22] = 2;
      put(tmp, c);
      run_file(tmp);
      c = w;
      c[34] = 24;
      put(tmp, c);
      run_file(tmp);
      c = w;   // data size larger than the file
      put_u32(c, 40, 0x7FFFFFF0u);
      put(tmp, c);
      run_file(tmp);
    }
  }
  // wk_augment over edge arguments (speed, volume, lengths)
  std::vector<float> in(1000), out(2000);
  for (size_t i = 0; i < in.size(); ++i) in[i] = 0.001f * (float)i - 0.5f;
  const float speeds[] = {1e-9f, 0.001f, 0.8f, 1.0f, 1.2f, 7.5f, 1e12f};
  const float vols[] = {0.7f, 1.0f, 1.3f, 1e30f};
  for (float sp : speeds)
    for (float vo : vols)
      for (int32_t n : {1, 2, 999, 1000})
        for (int32_t ol : {1, 1000, 2000}) (void)wk_augment(in.data(), n, sp, vo, 0.005f, 3u, out.data(), ol);
  printf("wav harness: %ld reads, %ld accepted\n", g_cases, g_ok);
  return 0;
}
