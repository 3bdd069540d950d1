/* Host-only ASan/UBSan harness for the C oracle (oracle/esp_mfcc_oracle.c) --
 * test infrastructure, built and run by tests/test_sanitizers.py on the CPU.
 * Runs the DFT path and the FFT batch path over parameter sets that reach its
 * edge cases: one-frame signals, frames longer than n_fft (truncated), more
 * coefficients than filters, a crowded filterbank with degenerate triangles
 * (0/0 weights), the 4096-point FFT, many threads, and the bad-argument
 * returns. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

int esp_mfcc_oracle_ex(const float* x, int L, int sr, int frame, int hop, int n_fft, int n_filters, int n_mfcc,
                       int esp_pack, float pre, float* out);
int esp_mfcc_oracle_batch(const float* x, long long n_clips, int L, long long stride, int sr, int frame, int hop,
                          int n_fft, int n_filters, int n_mfcc, int esp_pack, float pre, int n_threads, float* out);

int main(void) {
  const int cfg[][6] = {{16000, 320, 256, 512, 40, 13}, {8000, 200, 80, 256, 26, 12}, {16000, 512, 128, 256, 30, 13},
                        {16000, 320, 256, 512, 40, 45}, {4000, 100, 50, 128, 64, 13}, {44100, 2048, 441, 4096, 128, 40},
                        {16000, 1, 1, 2, 1, 1}};
  const int L = 5000;
  float* x = (float*)malloc(sizeof(float) * 3 * L);
  for (int i = 0; i < 3 * L; ++i) x[i] = 0.3f * sinf(0.01f * (float)i) + 0.01f * (float)((i * 7919) % 13 - 6);
  int runs = 0;
  for (unsigned c = 0; c < sizeof cfg / sizeof cfg[0]; ++c) {
    const int *p = cfg[c], len = p[1] <= L ? L : p[1];
    if (len > L) continue;
    const int nf = (len - p[1]) / p[2] + 1;
    float* o = (float*)malloc(sizeof(float) * (size_t)nf * p[5] * 3);
    for (int pack = 0; pack < 2; ++pack) {
      if (esp_mfcc_oracle_ex(x, len, p[0], p[1], p[2], p[3], p[4], p[5], pack, 0.97f, o) != nf) return 10 + (int)c;
      ++runs;
      if ((p[3] & (p[3] - 1)) == 0 && p[1] <= p[3] && p[5] <= p[4]) {
        if (esp_mfcc_oracle_batch(x, 3, len, L, p[0], p[1], p[2], p[3], p[4], p[5], pack, 0.97f, 3, o) != nf)
          return 30 + (int)c;
        ++runs;
      }
    }
    free(o);
  }
  float o1[64];
  if (esp_mfcc_oracle_ex(NULL, L, 16000, 320, 256, 512, 40, 13, 1, 0.97f, o1) != -1) return 50;
  if (esp_mfcc_oracle_ex(x, 100, 16000, 320, 256, 512, 40, 13, 1, 0.97f, o1) != -1) return 51;
  if (esp_mfcc_oracle_ex(x, L, 16000, 320, 0, 512, 40, 13, 1, 0.97f, o1) != -1) return 52;
  if (esp_mfcc_oracle_batch(x, 1, L, L, 16000, 320, 256, 500, 40, 13, 1, 0.97f, 1, o1) != -1) return 53;
  printf("oracle harness: %d runs\n", runs);
  free(x);
  return 0;
}
