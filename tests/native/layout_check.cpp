// Host-side check of the fused kernels' slab layout (csrc/kernels/lenet_layout.h), built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host (tests/test_native_host_cpu.py):
// for every grid / batch the kernels use, slab_off maps (slot, row) one-to-one onto
// [0, rows_total * 64) -- no two workgroups' writes collide and none leaves the buffer the
// engine allocates -- and slot_param / slab_slot are inverse on the parameters.
#include <cstdio>
#include <vector>

#include "kernels/lenet_layout.h"

using namespace csed::lenet;

static int check(int G, int B) {
  const int R2 = G < B ? G : B;
  const long total = (long)(C1_CH * G + (N_CHUNKS - C1_CH) * R2) * 64;  // the layout's span
  std::vector<unsigned char> hit(total, 0);
  int bad = 0;
  if (total > (long)G * CNP_PAD) {  // engine/fused.py allocates [grid, CNP_PAD]
    std::printf("G=%d B=%d span %ld exceeds the %ld-float allocation\n", G, B, total, (long)G * CNP_PAD);
    ++bad;
  }
  for (int s = 0; s < CNP_PAD; ++s) {
    const int rows = (s >> 6) < C1_CH ? G : R2;
    for (int r = 0; r < rows; ++r) {
      const int o = slab_off(s, r, G, R2);
      if (o < 0 || o >= total) {
        if (bad++ < 5) std::printf("G=%d B=%d slot %d row %d -> %d out of [0, %ld)\n", G, B, s, r, o, total);
        continue;
      }
      if (hit[o]++ && bad++ < 5) std::printf("G=%d B=%d slot %d row %d -> %d written twice\n", G, B, s, r, o);
    }
  }
  for (long i = 0; i < total; ++i)
    if (!hit[i] && bad++ < 5) std::printf("G=%d B=%d word %ld never written\n", G, B, i);
  return bad;
}

int main() {
  int bad = 0;
  for (int p = 0; p < CNP; ++p) {
    const int s = slab_slot(p);
    if (s < 0 || s >= CNP_PAD || slot_param(s) != p) {
      if (bad++ < 5) std::printf("param %d -> slot %d -> param %d\n", p, s, slot_param(s));
    }
  }
  int padding = 0;
  for (int s = 0; s < CNP_PAD; ++s) padding += slot_param(s) < 0;
  if (padding != CNP_PAD - CNP) {
    std::printf("padding slots %d, expected %d\n", padding, CNP_PAD - CNP);
    ++bad;
  }
  // split step (grid = SPLIT_K * B), one workgroup per sample, and the multi-sample grid 256
  for (int B : {1, 2, 3, 8, 16, 24, 32, 48, 64}) {
    bad += check(SPLIT_K * B, B);
    bad += check(B, B);
  }
  for (int B : {100, 256, 1000, 8192}) bad += check(256, B);
  std::printf(bad ? "layout check FAILED (%d)\n" : "layout check ok\n", bad);
  return bad ? 1 : 0;
}
