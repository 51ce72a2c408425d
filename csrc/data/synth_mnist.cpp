// Native synthetic-MNIST generator (host code, no torch, no GPU): the data-loading step of the
// benchmark and the CLIs, built as its own small shared object (_csed_data.so) so it can run
// BEFORE `import torch` -- in a thread that holds no Python lock -- and overlap the 1.4 s import.
//
// The recipe is data/mnist.py:synthetic_mnist's (a class-conditional stroke-prototype mixture,
// a confusable distractor, a random affine map composed with a smooth elastic field, bilinear
// resampling with zero padding, contrast, Gaussian-ish noise and salt), with its own
// counter-based random stream (SplitMix64 of (seed, split, sample, slot)) instead of torch's
// sequential generator: every sample is independent of every other, so the set is the same for
// any thread count.  The stroke prototypes come from the caller (data/native_synth.py computes
// them with numpy, as data/mnist.py does).
//
// The reference loads real MNIST with torchvision (ref src/train_dist.py:22-30); there is no
// network here, so this stands in for the dataset on disk.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

constexpr int kSide = 28, kPix = kSide * kSide, kStyles = 4;

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Uniform [0, 1) float from 24 random bits of stream (key, slot).
struct Stream {
  uint64_t key;
  inline float u(uint64_t slot) const { return (float)(splitmix64(key ^ (slot * 0xD1B54A32D192ED03ull)) >> 40) * (1.0f / 16777216.0f); }
  inline uint32_t bits(uint64_t slot) const { return (uint32_t)(splitmix64(key ^ (slot * 0xD1B54A32D192ED03ull)) >> 32); }
};

// 4 -> 28 linear interpolation weights, align_corners=True: output i sits at 3 i / 27 of the
// 4-point grid
struct Up {
  int lo[kSide];
  float w[kSide];
  Up() {
    for (int i = 0; i < kSide; ++i) {
      const float t = (float)i * 3.0f / 27.0f;
      int l = std::min((int)t, 2);
      lo[i] = l;
      w[i] = t - (float)l;
    }
  }
};

void make_sample(const float* protos, int classes, const Stream& st, const Up& up, uint8_t* img_out,
                 int64_t* label_out) {
  const int lab = (int)(st.bits(0) % (uint32_t)classes);
  float r[9];
  for (int j = 0; j < 9; ++j) r[j] = st.u(1 + j);
  const int style = std::min((int)(r[0] * kStyles), kStyles - 1);
  const int other = (lab + 1 + std::min((int)(r[1] * (classes - 1)), classes - 2)) % classes;
  const int ostyle = std::min((int)(r[2] * kStyles), kStyles - 1);
  const float* pa = protos + ((int64_t)lab * kStyles + style) * kPix;
  const float* pb = protos + ((int64_t)other * kStyles + ostyle) * kPix;
  const float dw = r[3] * 0.6f;
  // the blended source with a 2-pixel zero border: bilinear taps need no bounds checks (sample
  // coordinates are clamped to [-2, 28]: both taps of a clamped coordinate lie in the zero
  // border, so the clamp changes no output, and the right / lower tap of 28 is border index 31)
  constexpr int kP = kSide + 4;
  float src[kP * kP];
  std::fill(src, src + kP * kP, 0.0f);
  for (int y = 0; y < kSide; ++y)
    for (int x = 0; x < kSide; ++x) src[(y + 2) * kP + x + 2] = std::max(pa[y * kSide + x], pb[y * kSide + x] * dw);

  // affine map in normalised coordinates (1 px = 2/28) + elastic displacement (2 x 4 x 4 coarse
  // field, upsampled bilinearly to 28 x 28)
  const float ang = (r[4] - 0.5f) * 0.6f, sc = 0.8f + 0.4f * r[5], sh = (r[6] - 0.5f) * 0.3f;
  const float tx = (st.u(10) - 0.5f) * (12.0f / 28.0f), ty = (st.u(11) - 0.5f) * (12.0f / 28.0f);
  const float c = std::cos(ang) / sc, s = std::sin(ang) / sc;
  const float t00 = c, t01 = -s + sh, t10 = s, t11 = c;
  float coarse[2][4][4];
  for (int k = 0; k < 2; ++k)
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) coarse[k][a][b] = (st.u(12 + k * 16 + a * 4 + b) - 0.5f) * 0.16f;
  // rows of the field: coarse rows interpolated along x first (4 x 28 per component)
  float rowx[2][4][kSide];
  for (int k = 0; k < 2; ++k)
    for (int a = 0; a < 4; ++a)
      for (int x = 0; x < kSide; ++x)
        rowx[k][a][x] = coarse[k][a][up.lo[x]] * (1.0f - up.w[x]) + coarse[k][a][up.lo[x] + 1] * up.w[x];

  const float amp = 0.55f + 0.45f * r[7];
  // per-pixel noise: a PCG32 stream seeded from the sample's key (sequential within the sample)
  uint64_t pcg = st.key ^ 0x853C49E6748FEA9Bull;
  auto next_u = [&pcg]() {
    const uint64_t old = pcg;
    pcg = old * 6364136223846793005ull + 1442695040888963407ull;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u), rot = (uint32_t)(old >> 59u);
    const uint32_t v = (xs >> rot) | (xs << ((32u - rot) & 31u));
    return (float)(v >> 8) * (1.0f / 16777216.0f);
  };
  for (int y = 0; y < kSide; ++y) {
    const float cy = (float)(2 * y + 1) / kSide - 1.0f;
    const int ay = up.lo[y];
    const float wy = up.w[y];
    for (int x = 0; x < kSide; ++x) {
      const float cx = (float)(2 * x + 1) / kSide - 1.0f;
      const float ex = rowx[0][ay][x] * (1.0f - wy) + rowx[0][ay + 1][x] * wy;
      const float ey = rowx[1][ay][x] * (1.0f - wy) + rowx[1][ay + 1][x] * wy;
      const float gx = t00 * cx + t01 * cy + tx + ex;
      const float gy = t10 * cx + t11 * cy + ty + ey;
      // grid_sample, bilinear, zero padding, align_corners=False
      const float ix = std::min(std::max(((gx + 1.0f) * kSide - 1.0f) * 0.5f, -2.0f), 28.0f);
      const float iy = std::min(std::max(((gy + 1.0f) * kSide - 1.0f) * 0.5f, -2.0f), 28.0f);
      const float fx = std::floor(ix), fy = std::floor(iy);
      const int x0 = (int)fx + 2, y0 = (int)fy + 2;  // in the bordered image
      const float wx1 = ix - fx, wy1 = iy - fy, wx0 = 1.0f - wx1, wy0 = 1.0f - wy1;
      const float* q = src + y0 * kP + x0;
      float v = (q[0] * wx0 + q[1] * wx1) * wy0 + (q[kP] * wx0 + q[kP + 1] * wx1) * wy1;
      // contrast, noise of sigma 0.2 (a uniform of width 0.69) and sparse salt from one field
      const float uu = next_u();
      v = std::max(v * amp + (uu - 0.5f) * 0.69f, 0.0f) + std::max(uu - 0.98f, 0.0f) * 50.0f;
      v = std::min(std::max(v * 255.0f, 0.0f), 255.0f);
      img_out[y * kSide + x] = (uint8_t)v;  // truncation, as a float -> uint8 tensor copy
    }
  }
  *label_out = lab;
}

}  // namespace

extern "C" {

// images: uint8 [n][28][28], labels: int64 [n]; protos: float32 [classes][4][28][28] in [0, 1].
// Returns 0 on success.
int csed_synth_mnist(const float* protos, int classes, int64_t n, uint64_t seed, int train, uint8_t* images,
                     int64_t* labels, int threads) {
  if (!protos || !images || !labels || n < 0 || classes < 2) return 1;
  const Up up;
  const uint64_t base = splitmix64(seed * 2 + (train ? 0 : 1) + 0x5EEDull);
  threads = std::max(1, std::min(threads, 64));
  auto work = [&](int t) {
    for (int64_t i = t; i < n; i += threads) {
      const Stream st{splitmix64(base ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull))};
      make_sample(protos, classes, st, up, images + i * kPix, labels + i);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  return 0;
}

}  // extern "C"
