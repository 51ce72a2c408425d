// Fused LeNet (ref src/model.py:4-22) training step for gfx950.
//
// One workgroup (512 threads = 8 waves, two per SIMD) owns whole samples: it
// gathers the raw uint8 image, normalises it, runs conv1 -> pool -> relu ->
// conv2 -> Dropout2d -> pool -> relu -> fc1 -> relu -> dropout -> fc2 ->
// log_softmax -> NLL, and the complete backward pass, with every activation
// resident in LDS.  The only global traffic per sample is the 784-byte image;
// per workgroup it is the 33 KB of conv weight images (to LDS), the fc1
// fragments (to registers, reused across samples) and the partial gradient
// (21,840 fp32) written once to a slab.  A second kernel (lenet_update)
// reduces the slabs in a fixed order, applies SGD with momentum, refreshes
// the 16-bit weight images and bumps the device step/cursor/RNG counters, so
// a training step is exactly two launches (plus one RCCL all-reduce between
// them for DDP).
//
// Matrix work runs on v_mfma_f32_16x16x32_{bf16,f16}:
//   conv1 fwd   : [576 px x 25] . [25 x 10]        36 tiles, 1 K-step
//   conv2 fwd   : [64 px x 250] . [250 x 20]       4x2 tiles, 8 K-steps (one tile per wave)
//   fc1 fwd     : [1 x 320] . [320 x 50]           4 tiles (row 0 live), 10 K-steps
//   fc1 dX      : 320 x 50 VALU dot products from the LDS F1 image
//   conv2 wgrad : [20 x 64 px] . [64 px x 251]     2x16 tiles (col 250 = bias grad)
//   conv2 dgrad : [144 px x 500] . [500 x 10]      9 tiles, 16 K-steps (tile 8 split over waves)
//   conv1 wgrad : [10 x 576 px] . [576 px x 26]    1x2 tiles (col 25 = bias grad), 18 K-steps
// im2col operands are gathered from LDS through int16 k->offset tables read
// 8 at a time (ds_read_b128), so a gathered fragment costs 1 + 8 LDS reads
// and no integer division.  The pool-fused pixel order (m = 4*window +
// dy*2+dx) puts each 2x2 window in one lane's four accumulators (C row =
// 4*(lane>>4) + reg): max-pool, argmax, bias, ReLU and the Dropout2d scale
// are register-only epilogues.
//
// Weight-image layout (16-bit, offsets in elements; all 16-B aligned):
//   W1C  [16][32]   conv1  B operand  (k = kh*5+kw)
//   W2C  [32][264]  conv2  B operand  (k = ic*25+kh*5+kw), padded rows
//   W2D  [16][520]  conv2 dgrad B     (k' = oc*25 + (4-kh)*5 + (4-kw))
//   F1   [64][328]  fc1 B operand     (rows = out features)
//   F1T  [320][72]  reserved (fc1 dX runs on the VALU from the F1 image in LDS)
// fp32 values used as-is from the flat parameter buffer: all biases and fc2.
//
// Flat parameter order (= Net.state_dict() order, 21,840 floats):
//   conv1.w 0, conv1.b 250, conv2.w 260, conv2.b 5260, fc1.w 5280,
//   fc1.b 21280, fc2.w 21330, fc2.b 21830.
#include "common.h"
#include "dispatch.h"

namespace csed {

namespace lenet {
constexpr int NP = 21840;
constexpr int O_C1W = 0, O_C1B = 250, O_C2W = 260, O_C2B = 5260, O_F1W = 5280, O_F1B = 21280,
              O_F2W = 21330, O_F2B = 21830;
constexpr int I_W1C = 0, I_W2C = 512, I_W2D = 8960, I_F1 = 17280, I_F1T = 38272, I_END = 61312;
constexpr int LD_W2C = 264, LD_W2D = 520, LD_F1 = 328, LD_F1T = 72;
constexpr int LD_DC2 = 72, LD_DC1 = 584;
constexpr int NT = 512, NW = 8;
// conv partial-gradient slab: params [0, CNP) = conv1.w, conv1.b, conv2.w, conv2.b
constexpr int CNP = O_F1W;
constexpr int CNP_PAD = (CNP + 63) / 64 * 64;  // slab row: 83 chunks of 64 floats (see lenet_update)
// per-sample vector slab (fp32): fc1 input P2 | dL/dz1 | fc1 output H | dL/dlogits
constexpr int V_P2 = 0, V_DZ1 = 320, V_H = 384, V_DLOG = 448, VEC = 464;

// LDS carve (bytes); every region 16-B aligned
constexpr int S_W2C = 0;                              // u16 32*264
constexpr int S_W2D = S_W2C + 32 * LD_W2C * 2;        // u16 16*520
constexpr int S_F1 = S_W2D + 16 * LD_W2D * 2;         // u16 64*328 fc1 weight image
// W2C | W2D | F1 are contiguous here exactly as in the global image: one flat copy
constexpr int WIMG_LDS_U4 = (I_F1T - I_W2C) / 8;      // 16-byte vectors to stage
constexpr int S_X = S_F1 + 64 * LD_F1 * 2;            // u16 784 (+16 pad)
constexpr int S_P1 = S_X + 800 * 2;                   // u16 1440   [ic][12][12]
constexpr int S_I1 = S_P1 + 1440 * 2;                 // u8 1440    argmax in window
constexpr int S_P2 = S_I1 + 1440;                     // u16 320    [oc][4][4] = fc1 input
constexpr int S_I2 = S_P2 + 320 * 2;                  // u8 320
constexpr int S_DC2 = S_I2 + 320;                     // u16 32*72  dL/dconv2 [oc][pix]
constexpr int S_DC2P = S_DC2 + 32 * LD_DC2 * 2;       // u16 20*256 same, zero-padded [oc][16][16]
constexpr int S_DC1 = S_DC2P + 20 * 256 * 2;          // u16 16*584 dL/dconv1 [oc][pix]
constexpr int S_KO2 = S_DC1 + 16 * LD_DC1 * 2;        // i16 256    conv2 k -> P1 offset
constexpr int S_KOD = S_KO2 + 256 * 2;                // i16 512    dgrad k' -> DC2P offset
constexpr int S_DZ1B = S_KOD + 512 * 2;               // u16 64     dZ1 as the MFMA A row
constexpr int S_F = S_DZ1B + 64 * 2;                  // f32 scratch
constexpr int F_D2S = 0, F_D1S = 32, F_H = 96, F_DLOG = 160, F_DZ1 = 176, F_DP2 = 240, F_PAR = 560,
              F_RED = 1152, F_LAB = 3200, F_END = 3204;
// fp32 params cached in LDS (offsets inside F_PAR): c1b 0, c2b 10, f1b 30, f2b 80, f2w 90 (500) -> 590
constexpr int P_C1B = 0, P_C2B = 10, P_F1B = 30, P_F2B = 80, P_F2W = 90;
constexpr int S_TOTAL = S_F + F_END * 4;
static_assert(S_W2D % 16 == 0 && S_X % 16 == 0 && S_P1 % 16 == 0 && S_I1 % 16 == 0, "align");
static_assert(S_P2 % 16 == 0 && S_I2 % 16 == 0 && S_DC2 % 16 == 0 && S_DC2P % 16 == 0, "align");
static_assert(S_DC1 % 16 == 0 && S_KO2 % 16 == 0 && S_KOD % 16 == 0 && S_DZ1B % 16 == 0, "align");
static_assert(S_F % 16 == 0 && S_TOTAL <= 160 * 1024, "lds");
static_assert(S_W2D == (I_W2D - I_W2C) * 2 && S_F1 == (I_F1 - I_W2C) * 2, "LDS image must mirror wimg");
}  // namespace lenet

using namespace lenet;

typedef short s16x8 __attribute__((ext_vector_type(8)));

// Diagnostic stage stamps (a.dbg non-null): thread 0 of each workgroup records
// s_memtime at each stage start of its first sample.  Only for profiling builds
// of the step; read the shares, not the absolute time.
#define STAMP(i)                                                              \
  do {                                                                        \
    if (a.dbg && tid == 0 && s == 0) a.dbg[g * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

template <typename T>
__device__ __forceinline__ unsigned short h16(float v) { return bits_of<T>((T)v); }
template <typename T>
__device__ __forceinline__ float f16v(unsigned short b) { return (float)of_bits<T>(b); }

// conv2 dgrad epilogue for one (input channel, P1 pixel): relu gate, then the
// pool1 backward scatter of the 2x2 window (argmax position gets the value).
template <typename T>
__device__ __forceinline__ void dgrad_out(unsigned short* DC1, const unsigned short* P1, const uint8_t* I1,
                                          int ci, int mm, float v) {
  const int ih = mm / 12, iw = mm - ih * 12;
  const int pi = ci * 144 + mm;
  v = f16v<T>(P1[pi]) > 0.f ? v : 0.f;
  const int bi = I1[pi];
  unsigned short* d = DC1 + ci * LD_DC1 + (2 * ih) * 24 + 2 * iw;
  const unsigned short hv = h16<T>(v), z = 0;
  d[0] = bi == 0 ? hv : z;
  d[1] = bi == 1 ? hv : z;
  d[24] = bi == 2 ? hv : z;
  d[25] = bi == 3 ? hv : z;
}

template <typename T, bool TRAIN>
__global__ void __launch_bounds__(NT, 2) lenet_train_kernel(LenetTrainArgs a, int write_logp, float* logp_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  typedef typename Mfma<T>::frag frag;
  unsigned short* W2c = (unsigned short*)(sm + S_W2C);
  unsigned short* W2d = (unsigned short*)(sm + S_W2D);
  unsigned short* Xs = (unsigned short*)(sm + S_X);
  unsigned short* P1 = (unsigned short*)(sm + S_P1);
  uint8_t* I1 = sm + S_I1;
  unsigned short* P2 = (unsigned short*)(sm + S_P2);
  uint8_t* I2 = sm + S_I2;
  unsigned short* DC2 = (unsigned short*)(sm + S_DC2);
  unsigned short* DC2P = (unsigned short*)(sm + S_DC2P);
  unsigned short* DC1 = (unsigned short*)(sm + S_DC1);
  short* KO2 = (short*)(sm + S_KO2);
  short* KOD = (short*)(sm + S_KOD);
  unsigned short* DZ1B = (unsigned short*)(sm + S_DZ1B);
  unsigned short* F1s = (unsigned short*)(sm + S_F1);
  float* Fs = (float*)(sm + S_F);
  float* D2S = Fs + F_D2S;
  float* D1S = Fs + F_D1S;
  float* Hs = Fs + F_H;
  float* DLOG = Fs + F_DLOG;
  float* DZ1 = Fs + F_DZ1;
  float* DP2 = Fs + F_DP2;
  float* PAR = Fs + F_PAR;
  float* RED = Fs + F_RED;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kb = 8 * (lane >> 4);
  const int G = gridDim.x, g = blockIdx.x;
  const float inv_std = 1.f / a.std_;
  const uint64_t rng_off = TRAIN ? rng_offset(0, a.rng_offset) : 0;
  const frag zfrag = __builtin_bit_cast(frag, u16x8{0, 0, 0, 0, 0, 0, 0, 0});

  if (a.dbg && tid == 0) a.dbg[g * 16 + 12] = __builtin_amdgcn_s_memtime();
  // ---------------- once per workgroup: weight images, offset tables, fp32 params -> LDS
  // register-resident conv1 weight fragment, reused for every sample of this WG
  frag fb1;
  {
    // Every global load of the preamble (weight images, fp32 params, the conv1
    // fragment) is issued before the first wait: one memory round trip.
    constexpr int PER = (WIMG_LDS_U4 + NT - 1) / NT;
    const uint4* src = reinterpret_cast<const uint4*>(a.wimg + I_W2C);
    uint4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) v[u] = src[min(tid + u * NT, WIMG_LDS_U4 - 1)];  // unconditional: no branches
    // fp32 params: c1b, c2b, f1b, f2b, f2w (590 floats, one per thread)
    int pi = O_F2W + tid - 90;
    if (tid < 10) pi = O_C1B + tid;
    else if (tid < 30) pi = O_C2B + tid - 10;
    else if (tid < 80) pi = O_F1B + tid - 30;
    else if (tid < 90) pi = O_F2B + tid - 80;
    const float pv0 = a.params[pi];
    const float pv1 = a.params[O_F2W + min(tid + NT, 589) - 90];
    fb1 = *reinterpret_cast<const frag*>(a.wimg + I_W1C + l16 * 32 + kb);
    // work that needs no loaded data overlaps the loads
    if (tid < 256) {
      const int k = tid, ic = k / 25, r = k % 25;
      KO2[k] = (short)(k < 250 ? ic * 144 + (r / 5) * 12 + (r % 5) : 0);
    }
    {
      const int k = tid, co = k / 25, r = k % 25;
      KOD[k] = (short)(k < 500 ? co * 256 + (r / 5) * 16 + (r % 5) : 0);
    }
    // DC2 | DC2P | DC1 are contiguous: zero their padding once with 16-B stores
    {
      constexpr int NZ = (S_KO2 - S_DC2) / 16;
      uint4* z = reinterpret_cast<uint4*>(sm + S_DC2);
      for (int i = tid; i < NZ; i += NT) z[i] = make_uint4(0, 0, 0, 0);
    }
    uint4* dst = reinterpret_cast<uint4*>(W2c);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int i = tid + u * NT;
      if (i < WIMG_LDS_U4) dst[i] = v[u];
    }
    if (tid < 590) PAR[tid] = pv0;
    if (tid + NT < 590) PAR[tid + NT] = pv1;
  }
  if (a.dbg && tid == 0) a.dbg[g * 16 + 13] = __builtin_amdgcn_s_memtime();
  if (a.dbg && tid == 0) a.dbg[g * 16 + 14] = __builtin_amdgcn_s_memtime();
  int koff1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kb + j;
    koff1[j] = k < 25 ? (k / 5) * 28 + (k % 5) : 0;
  }

  // ---------------- per-workgroup gradient accumulators (registers)
  f32x4 acc_c2[2][2];   // conv2 wgrad: M-tiles (oc) 0,1 x N-tiles (k) wave, wave+8
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc_c2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc_c1 = f32x4{0.f, 0.f, 0.f, 0.f};  // conv1 wgrad tile (wave&1), steps (wave>>1) mod 4
  float loss_sum = 0.f, correct = 0.f;
  // The fc-layer weight gradients are rank-1 per sample (dZ (x) input); instead of
  // accumulating 16,500 products per sample here, each sample's vectors are written
  // to the vector slab and lenet_update forms the sums as one GEMM over the batch.

  const int nsamp = (a.B - g + G - 1) / G;
  for (int s = 0; s < nsamp; ++s) {
    const int b = g + s * G;
    float* vs = TRAIN ? a.vslab + (int64_t)b * VEC : nullptr;
    __syncthreads();  // previous sample's readers of Xs / P1 / DC1 are done
    // ---------------- stage 0: gather + normalise the image, dropout masks
    STAMP(0);
    const int64_t row = a.perm[(a.cursor ? a.cursor[0] : 0) * (int64_t)a.B + b];
    {
      const uint8_t* img = a.images + row * 784;
      for (int i = tid; i < 784; i += NT) Xs[i] = h16<T>(((float)img[i] * (1.f / 255.f) - a.mean) * inv_std);
      if (tid < 70) {
        float sc = 1.f;
        if (TRAIN) {
          const uint64_t e = (uint64_t)(a.rank_stride * (int64_t)a.B + b) * 70ull + tid;
          sc = dropout_keep(a.seed, rng_off, e, a.drop_p) ? 1.f / (1.f - a.drop_p) : 0.f;
        }
        if (tid < 20) D2S[tid] = sc;
        else D1S[tid - 20] = sc;
      }
      if (tid == 0) Fs[F_LAB] = __int_as_float((int)a.labels[row]);
    }
    __syncthreads();

    // ---------------- stage 1: conv1 + bias + maxpool + relu -> P1, I1
    STAMP(1);
#pragma unroll
    for (int it = 0; it < 5; ++it) {  // 36 tiles over 8 waves, unrolled so all gathers issue up front
      const int mt = wave + it * NW;
      if (mt >= 36) break;
      const int m = mt * 16 + l16;
      const int p = m >> 2, q = m & 3;
      const int pb = (2 * (p / 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1);
      u16x8 raw;
#pragma unroll
      for (int j = 0; j < 8; ++j) raw[j] = Xs[pb + koff1[j]];
      const f32x4 c = Mfma<T>::mma(__builtin_bit_cast(frag, raw), fb1, f32x4{0.f, 0.f, 0.f, 0.f});
      if (l16 < 10) {
        float best = c[0];
        int bi = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (c[r] > best) { best = c[r]; bi = r; }
        const int w = mt * 4 + (lane >> 4);
        P1[l16 * 144 + w] = h16<T>(fmaxf(best + PAR[P_C1B + l16], 0.f));
        I1[l16 * 144 + w] = (uint8_t)bi;
      }
    }
    __syncthreads();

    // ---------------- stage 2: conv2 + bias + Dropout2d + maxpool + relu -> P2, I2
    STAMP(2);
    {
      const int mt = wave & 3, nt = wave >> 2;
      const int m = mt * 16 + l16;
      const int p = m >> 2, q = m & 3;
      const int pb = (2 * (p >> 2) + (q >> 1)) * 12 + 2 * (p & 3) + (q & 1);
      f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
      const unsigned short* wrow = W2c + (nt * 16 + l16) * LD_W2C + kb;
#pragma unroll 4
      for (int ks = 0; ks < 8; ++ks) {
        const s16x8 o = *reinterpret_cast<const s16x8*>(KO2 + ks * 32 + kb);
        u16x8 raw;
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[j] = P1[pb + o[j]];
        c = Mfma<T>::mma(__builtin_bit_cast(frag, raw), *reinterpret_cast<const frag*>(wrow + ks * 32), c);
      }
      const int oc = nt * 16 + l16;
      if (oc < 20) {
        float best = c[0];
        int bi = 0;
#pragma unroll
        for (int r = 1; r < 4; ++r)
          if (c[r] > best) { best = c[r]; bi = r; }
        const int w = mt * 4 + (lane >> 4);
        const unsigned short hv = h16<T>(fmaxf(best + PAR[P_C2B + oc], 0.f) * D2S[oc]);
        P2[oc * 16 + w] = hv;
        I2[oc * 16 + w] = (uint8_t)bi;
        if (TRAIN) vs[V_P2 + oc * 16 + w] = f16v<T>(hv);  // fc1 input, exactly as the forward used it
      }
    }
    __syncthreads();

    // ---------------- stage 3: fc1 + bias + relu + dropout -> H   (waves 0-3)
    STAMP(3);
    if (wave < 4) {
      f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
      const unsigned short* wrow = F1s + (wave * 16 + l16) * LD_F1 + kb;
#pragma unroll 5
      for (int ks = 0; ks < 10; ++ks) {
        const frag fa = l16 == 0 ? *reinterpret_cast<const frag*>(P2 + ks * 32 + kb) : zfrag;
        c = Mfma<T>::mma(fa, *reinterpret_cast<const frag*>(wrow + ks * 32), c);
      }
      if (lane < 16) {
        const int o = wave * 16 + lane;
        if (o < 50) {
          const float h = fmaxf(c[0] + PAR[P_F1B + o], 0.f) * D1S[o];
          Hs[o] = h;
          if (TRAIN) vs[V_H + o] = h;
        }
      }
    }
    __syncthreads();

    // ---------------- stage 4: fc2 + log_softmax + NLL + dlogits (wave 0)
    STAMP(4);
    if (wave == 0) {
      const int t = __float_as_int(Fs[F_LAB]);
      // 4 lanes per logit (lanes 4c..4c+3 cover o = 13q .. 13q+12), then a
      // fixed-order 2-step butterfly inside each aligned 4-lane group
      float zp = 0.f;
      if (lane < 40) {
        const int c = lane >> 2, q = lane & 3;
        const float* wr = PAR + P_F2W + c * 50;
#pragma unroll
        for (int u = 0; u < 13; ++u) {
          const int o = q * 13 + u;
          if (o < 50) zp = fmaf(wr[o], Hs[o], zp);
        }
      }
      zp += __shfl_xor(zp, 1, 64);
      zp += __shfl_xor(zp, 2, 64);
      const float zc = __shfl(zp, (lane & 15) * 4, 64);
      const float logit = lane < 10 ? zc + PAR[P_F2B + lane] : -INFINITY;
      const float mx = wave_max(logit);
      const float e = lane < 10 ? __expf(logit - mx) : 0.f;
      const float se = wave_sum(e);
      const float lse = mx + __logf(se);
      const float lp = logit - lse;
      // first index attaining the max (torch argmax tie rule)
      const unsigned long long ismax = __ballot(lane < 10 && logit == mx);
      const int amax = __ffsll((long long)ismax) - 1;
      const float lt = __shfl(lp, t, 64);
      if (lane == 0) {
        loss_sum += -lt;
        correct += (amax == t) ? 1.f : 0.f;
      }
      if (write_logp && lane < 10) logp_out[(int64_t)b * 10 + lane] = lp;
      if (TRAIN && lane < 16) {
        const float dl = lane < 10 ? (__expf(lp) - (lane == t ? 1.f : 0.f)) * a.grad_scale : 0.f;
        DLOG[lane] = dl;
        vs[V_DLOG + lane] = dl;
      }
    }
    if (!TRAIN) continue;
    __syncthreads();

    // ---------------- stage 5: fc2 backward, fc1 relu/dropout gate
    STAMP(5);
    {
      if (tid < 64) {
        float dz = 0.f;
        if (tid < 50) {
          float dh = 0.f;
#pragma unroll
          for (int c = 0; c < 10; ++c) dh = fmaf(DLOG[c], PAR[P_F2W + c * 50 + tid], dh);
          dz = Hs[tid] > 0.f ? dh * D1S[tid] : 0.f;
          vs[V_DZ1 + tid] = dz;
        }
        DZ1[tid] = dz;
      }
    }
    __syncthreads();

    // ---------------- stage 6: dP2 = W1^T dZ1 (VALU over the LDS fc1 image)
    STAMP(6);
    {
      // dP2[i] = sum_o dZ1[o] * W1[o][i]: one input feature per thread, lanes read
      // consecutive columns of the LDS fc1 image (conflict-free), 50-long FMA chain
      if (tid < 320) {
        float d[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
        const unsigned short* col = F1s + tid;
#pragma unroll
        for (int o = 0; o < 50; ++o) d[o % 5] = fmaf(DZ1[o], f16v<T>(col[o * LD_F1]), d[o % 5]);
        DP2[tid] = ((d[0] + d[1]) + (d[2] + d[3])) + d[4];
      }
    }
    __syncthreads();

    // ---------------- stage 7: pool2 / relu / Dropout2d backward -> dC2 (two layouts)
    STAMP(7);
    for (int i = tid; i < 1280; i += NT) {
      const int oc = i >> 6, pix = i & 63;
      const int oh = pix >> 3, ow = pix & 7;
      const int w = (oh >> 1) * 4 + (ow >> 1);
      const int pos = (oh & 1) * 2 + (ow & 1);
      const int pi = oc * 16 + w;
      const float gv = (I2[pi] == pos && f16v<T>(P2[pi]) > 0.f) ? DP2[pi] * D2S[oc] : 0.f;
      const unsigned short hb = h16<T>(gv);
      DC2[oc * LD_DC2 + pix] = hb;
      DC2P[oc * 256 + (oh + 4) * 16 + (ow + 4)] = hb;
    }
    __syncthreads();

    // ---------------- stage 8: conv2 wgrad (+bias column 250), accumulate in registers
    STAMP(8);
    {
      const unsigned short one = h16<T>(1.f);
#pragma unroll
      for (int ps = 0; ps < 2; ++ps) {
        const frag fa0 = *reinterpret_cast<const frag*>(DC2 + l16 * LD_DC2 + ps * 32 + kb);
        const frag fa1 = *reinterpret_cast<const frag*>(DC2 + (16 + l16) * LD_DC2 + ps * 32 + kb);
        const int ohr = ((ps * 32 + kb) >> 3) * 12;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int k = (wave + 8 * jj) * 16 + l16;
          u16x8 raw;
          if (k < 250) {
            const int base = KO2[k] + ohr;
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[j] = P1[base + j];
          } else {
            const unsigned short v = k == 250 ? one : (unsigned short)0;
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[j] = v;
          }
          const frag fb = __builtin_bit_cast(frag, raw);
          acc_c2[0][jj] = Mfma<T>::mma(fa0, fb, acc_c2[0][jj]);
          acc_c2[1][jj] = Mfma<T>::mma(fa1, fb, acc_c2[1][jj]);
        }
      }
    }
    // ---------------- stage 9: conv2 dgrad -> dP1 -> relu/pool1 backward -> dC1
    STAMP(9);
    {
      const unsigned short* wrow = W2d + l16 * LD_W2D + kb;
      // full tile `wave` (pixels 16*wave .. +15)
      {
        const int m = wave * 16 + l16;
        const int pb = (m / 12) * 16 + (m % 12);
        f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
        for (int ks = 0; ks < 16; ++ks) {
          const s16x8 o = *reinterpret_cast<const s16x8*>(KOD + ks * 32 + kb);
          u16x8 raw;
#pragma unroll
          for (int j = 0; j < 8; ++j) raw[j] = DC2P[pb + o[j]];
          c = Mfma<T>::mma(__builtin_bit_cast(frag, raw), *reinterpret_cast<const frag*>(wrow + ks * 32), c);
        }
        if (l16 < 10) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dgrad_out<T>(DC1, P1, I1, l16, wave * 16 + 4 * (lane >> 4) + r, c[r]);
        }
      }
      // tile 8 (pixels 128..143): K-steps 2*wave, 2*wave+1 here, reduced below
      {
        const int m = 128 + l16;
        const int pb = (m / 12) * 16 + (m % 12);
        f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int ks = 2 * wave + kk;
          const s16x8 o = *reinterpret_cast<const s16x8*>(KOD + ks * 32 + kb);
          u16x8 raw;
#pragma unroll
          for (int j = 0; j < 8; ++j) raw[j] = DC2P[pb + o[j]];
          c = Mfma<T>::mma(__builtin_bit_cast(frag, raw), *reinterpret_cast<const frag*>(wrow + ks * 32), c);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) RED[wave * 256 + (4 * (lane >> 4) + r) * 16 + l16] = c[r];
      }
    }
    __syncthreads();
    if (tid < 256) {
      const int rr = tid >> 4, ci = tid & 15;
      if (ci < 10) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) v += RED[q * 256 + rr * 16 + ci];
        dgrad_out<T>(DC1, P1, I1, ci, 128 + rr, v);
      }
    }
    __syncthreads();

    // ---------------- stage 10: conv1 wgrad (+bias column 25), accumulate in registers
    STAMP(10);
    {
      const int nt = wave & 1;
      const int k = nt * 16 + l16;
      const unsigned short one = h16<T>(1.f);
      const int koff = k < 25 ? (k / 5) * 28 + (k % 5) : 0;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int ps = (wave >> 1) + 4 * i;
        if (ps < 18) {
          const int p0 = ps * 32 + kb;
          const frag fa = *reinterpret_cast<const frag*>(DC1 + l16 * LD_DC1 + p0);
          const int oh = p0 / 24, ow0 = p0 - oh * 24;
          u16x8 raw;
          if (k < 25) {
            const int base = oh * 28 + ow0 + koff;
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[j] = Xs[base + j];
          } else {
            const unsigned short v = k == 25 ? one : (unsigned short)0;
#pragma unroll
            for (int j = 0; j < 8; ++j) raw[j] = v;
          }
          acc_c1 = Mfma<T>::mma(fa, __builtin_bit_cast(frag, raw), acc_c1);
        }
      }
    }
  }

  {
    const int s = 0;
    STAMP(11);
  }
  // ---------------- epilogue: write this workgroup's partial gradient + loss
  if (TRAIN) {
    // slab layout: 64-float chunks of the conv gradient, workgroup-major inside a
    // chunk ([chunk][WG][64]) so lenet_update reads each chunk contiguously
    auto out = [&](int e) -> float& { return a.slab[((int64_t)(e >> 6) * G + g) * 64 + (e & 63)]; };
    // conv1: combine the four step-slices of each tile (fixed order)
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) RED[(wave * 16 + 4 * (lane >> 4) + r) * 16 + l16] = acc_c1[r];
    __syncthreads();
    {
      const int nt = tid >> 8, oc = (tid >> 4) & 15, col = tid & 15;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) v += RED[((nt + 2 * q) * 16 + oc) * 16 + col];
      const int k = nt * 16 + col;
      if (oc < 10) {
        if (k < 25) out(O_C1W + oc * 25 + k) = v;
        else if (k == 25) out(O_C1B + oc) = v;
      }
    }
    // conv2
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int k = (wave + 8 * jj) * 16 + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int oc = mt * 16 + 4 * (lane >> 4) + r;
          if (oc < 20) {
            if (k < 250) out(O_C2W + oc * 250 + k) = acc_c2[mt][jj][r];
            else if (k == 250) out(O_C2B + oc) = acc_c2[mt][jj][r];
          }
        }
      }
  }
  if (tid == 0) {
    a.loss_acc[2 * g] = loss_sum;
    a.loss_acc[2 * g + 1] = correct;
  }
}

// ---------------------------------------------------------------------------
// Weight images from fp32 params (element i of the flat buffer).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void write_images(unsigned short* wimg, int i, float v) {
  const unsigned short h = h16<T>(v);
  if (i < O_C1B) {
    wimg[I_W1C + (i / 25) * 32 + (i % 25)] = h;
  } else if (i >= O_C2W && i < O_C2B) {
    const int j = i - O_C2W;
    const int oc = j / 250, k = j % 250;
    wimg[I_W2C + oc * LD_W2C + k] = h;
    const int ic = k / 25, r = k % 25, kh = r / 5, kw = r % 5;
    wimg[I_W2D + ic * LD_W2D + oc * 25 + (4 - kh) * 5 + (4 - kw)] = h;
  } else if (i >= O_F1W && i < O_F1B) {
    const int j = i - O_F1W;
    const int o = j / 320, ii = j % 320;
    wimg[I_F1 + o * LD_F1 + ii] = h;
  }
}

template <typename T>
__global__ void lenet_pack_kernel(const float* __restrict__ params, unsigned short* __restrict__ wimg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NP) write_images<T>(wimg, i, params[i]);
}

// ---------------------------------------------------------------------------
// lenet_update: turn the step's partials into the gradient, then either
// export it (DDP: the RCCL all-reduce runs next) or apply SGD + refresh the
// 16-bit weight images.  Two block roles in one launch:
//
//   role CONV (blocks [0, NB_CONV)): fixed-order reduction of the per-WG conv
//     slabs, 16 float4 columns x 32 slices per block so every CU pulls only a
//     few KB with all loads in flight (latency-, not bandwidth-bound).  Block 0
//     also folds the loss partials and bumps the device counters.
//   role FC (blocks [NB_CONV, +NB_FC)): the fc gradients are batch GEMMs of the
//     per-sample vectors, on the fp32 MFMA (v_mfma_f32_16x16x4_f32, exact fp32
//     products), one 16x16 output tile per wave, K = batch:
//       dW1 | db1 = dZ1^T . [P2 | 1]   (4 x 21 tiles: column 320 = bias grad)
//       dW2 | db2 = dL^T  . [H  | 1]   (1 x 4 tiles:  column 50  = bias grad)
//     Each lane issues all of a 64-sample chunk's loads before its 16 MFMAs.
//
// Reductions run in a fixed order everywhere: bitwise reproducible.
// ---------------------------------------------------------------------------
constexpr int UP_C = 16, UP_S = 32, UP_MAXL = 8, UP_NT = UP_C * UP_S;
constexpr int CNQ = CNP / 4;                        // conv float4 columns (1320)
constexpr int NB_CONV = (CNQ + UP_C - 1) / UP_C;    // 83
constexpr int FC1_TILES = 4 * 21, FC_TILES = FC1_TILES + 4;
constexpr int NB_FC = (FC_TILES + UP_NT / 64 - 1) / (UP_NT / 64);  // 11 blocks x 8 waves
constexpr int NB_UPDATE = NB_CONV + NB_FC;

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

// Final consumer of one parameter's gradient: export or SGD step.  p / m are
// params[i] / momentum[i], loaded by the caller at kernel entry so their
// round trip overlaps the gradient loads instead of following them.
template <typename T>
__device__ __forceinline__ void finish_param(const LenetUpdateArgs& a, int i, float gsum, bool first, float p,
                                             float m) {
  if (!a.apply_sgd) {
    a.grad_out[i] = gsum;
    return;
  }
  if (a.grad_out) a.grad_out[i] = gsum;
  const float gj = gsum + a.weight_decay * p;
  float d = gj;
  if (a.mom != 0.f) {
    const float bj = first ? gj : fmaf(a.mom, m, (1.f - a.dampening) * gj);
    a.momentum[i] = bj;
    d = a.nesterov ? fmaf(a.mom, bj, gj) : bj;
  }
  p = fmaf(-a.lr, d, p);
  a.params[i] = p;
  write_images<T>(a.wimg, i, p);
}

template <typename T>
__global__ void __launch_bounds__(UP_NT) lenet_update_kernel(LenetUpdateArgs a, const float* __restrict__ vslab,
                                                             int B, float* loss_parts, int nparts,
                                                             float* loss_acc) {
  __shared__ float4 part[UP_S][UP_C];
  __shared__ float part2[4][UP_C * 4];
  // with zero dampening a zero-initialised momentum buffer reproduces torch's
  // first-step rule exactly (buf = m*0 + g), so step[0] is only read otherwise
  const bool first = (a.step && a.dampening != 0.f) ? a.step[0] == 0 : false;
  const int tid = threadIdx.x, blk = blockIdx.x;
#define USTAMP(k) \
  if (a.dbg && tid == 0) a.dbg[blk * 8 + (k)] = __builtin_amdgcn_s_memrealtime();
  USTAMP(0);

  if (blk < NB_CONV) {
    // ---------------- role CONV
    const int cl = tid & (UP_C - 1), sl = tid / UP_C;
    // wave 0 owns params blk*64 + tid (16 float4 columns): prefetch p / m now
    const int pi = blk * (UP_C * 4) + tid;
    float p0 = 0.f, m0 = 0.f;
    if (a.apply_sgd && tid < 64) {
      p0 = a.params[min(pi, NP - 1)];
      m0 = a.momentum[min(pi, NP - 1)];
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // Loads are unconditional from a clamped address and masked afterwards: a
    // per-element "load or zero" select makes hipcc branch around every load
    // and wait vmcnt(0) each time (dependent round trips instead of one).
    // chunk blk of the slab is [WG][16 float4]: contiguous for this block
    const float4* sp = reinterpret_cast<const float4*>(a.slab) + (int64_t)blk * a.grid * UP_C + cl;
    for (int g0 = sl; g0 < a.grid; g0 += UP_S * UP_MAXL) {
      float4 v[UP_MAXL];
#pragma unroll
      for (int u = 0; u < UP_MAXL; ++u) v[u] = sp[(int64_t)min(g0 + u * UP_S, a.grid - 1) * UP_C];
#pragma unroll
      for (int u = 0; u < UP_MAXL; ++u)
        if (g0 + u * UP_S < a.grid) add4(acc, v[u]);
    }
    USTAMP(1);
    part[sl][cl] = acc;
    __syncthreads();
    USTAMP(2);
    if (sl < 4) {
      float4 t = part[sl * 8][cl];
#pragma unroll
      for (int q = 1; q < 8; ++q) add4(t, part[sl * 8 + q][cl]);
      *reinterpret_cast<float4*>(&part2[sl][4 * cl]) = t;
    }
    __syncthreads();
    USTAMP(3);
    if (tid < 64 && pi < CNP) {
      const float g = (part2[0][tid] + part2[1][tid]) + (part2[2][tid] + part2[3][tid]);
      finish_param<T>(a, pi, g, first, p0, m0);
    }
    USTAMP(4);
    if (blk == 0 && loss_parts && tid < 64) {
      // loss / accuracy partials: lane-strided sums, then a fixed butterfly
      float s0 = 0.f, s1 = 0.f;
      for (int q = tid; q < nparts; q += 64) {
        s0 += loss_parts[2 * q];
        s1 += loss_parts[2 * q + 1];
      }
      s0 = wave_sum(s0);
      s1 = wave_sum(s1);
      if (tid == 0) {
        loss_acc[0] += s0;
        loss_acc[1] += s1;
      }
    }
  } else {
    // ---------------- role FC: one 16x16 tile of [dW | db] per wave
    const int wave = tid >> 6, lane = tid & 63, l16 = lane & 15, kq = lane >> 4;
    const int tile = (blk - NB_CONV) * (UP_NT / 64) + wave;
    if (tile < FC_TILES) {
      const bool fc1 = tile < FC1_TILES;
      const int mt = fc1 ? tile / 21 : 0, nt = fc1 ? tile % 21 : tile - FC1_TILES;
      const int rows = fc1 ? 50 : 10, cols = fc1 ? 320 : 50;
      const int a_off = fc1 ? V_DZ1 : V_DLOG, b_off = fc1 ? V_P2 : V_H;
      const int o = mt * 16 + l16, i = nt * 16 + l16;  // A row (out feature) / B col (in feature)
      // this lane's 4 outputs (C rows 4*kq + r, column i) and their p / m
      int pidx[4];
      float pp[4] = {0.f, 0.f, 0.f, 0.f}, pm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int oo = mt * 16 + 4 * kq + r;
        pidx[r] = (oo < rows && i <= cols)
                      ? (fc1 ? (i < cols ? O_F1W + oo * 320 + i : O_F1B + oo)
                             : (i < cols ? O_F2W + oo * 50 + i : O_F2B + oo))
                      : -1;
        if (a.apply_sgd) {
          pp[r] = a.params[max(pidx[r], 0)];
          pm[r] = a.momentum[max(pidx[r], 0)];
        }
      }
      f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
      // K = batch; 16x16x4 f32 MFMA: lane holds A[o][s0 + 4u + kq] and B[s0 + 4u + kq][i]
      for (int s0 = 0; s0 < B; s0 += 64) {
        float av[16], bv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int s = s0 + 4 * u + kq;
          const bool ok = s < B;
          // unconditional loads from clamped addresses, masked after (see role CONV)
          const float* rowc = vslab + (int64_t)min(s, B - 1) * VEC;
          const float ra = rowc[a_off + min(o, rows - 1)];
          const float rb = rowc[b_off + min(i, cols - 1)];
          av[u] = (ok && o < rows) ? ra : 0.f;
          bv[u] = ok ? (i < cols ? rb : (i == cols ? 1.f : 0.f)) : 0.f;
        }
        // keep all 32 loads in flight before the first MFMA (otherwise the
        // scheduler interleaves them and waits on each pair in turn)
        __builtin_amdgcn_sched_barrier(0);
        USTAMP(1);
#pragma unroll
        for (int u = 0; u < 16; ++u) c = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], c, 0, 0, 0);
      }
      USTAMP(2);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (pidx[r] >= 0) finish_param<T>(a, pidx[r], c[r], first, pp[r], pm[r]);
      USTAMP(4);
    }
  }

  if (a.apply_sgd) {
    // Device counters.  cursor / rng_offset are never read by this kernel, so
    // one thread bumps them directly.  step[0] is read by every block only when
    // dampening != 0; then the last block to take a ticket bumps it.
    if (a.dampening != 0.f) {
      __syncthreads();
      if (tid == 0) {
        const int t = atomicAdd(a.ticket, 1);  // every block read step[0] before this
        if (t == (int)gridDim.x - 1) {
          a.ticket[0] = 0;
          if (a.step) a.step[0] += 1;
        }
      }
    } else if (blk == 0 && tid == 0 && a.step) {
      a.step[0] += 1;
    }
    if (blk == 0 && tid == 0) {
      if (a.cursor) a.cursor[0] += 1;
      if (a.rng_offset) a.rng_offset[0] += 1;
    }
  }
}

// SGD from an already-reduced gradient (DDP: after the all-reduce).
template <typename T>
__global__ void lenet_sgd_kernel(LenetUpdateArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool first = (a.step && a.dampening != 0.f) ? a.step[0] == 0 : false;
  if (i < NP) finish_param<T>(a, i, a.grad_in[i], first, a.params[i], a.momentum[i]);
  if (a.dampening != 0.f) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const int t = atomicAdd(a.ticket, 1);
      if (t == (int)gridDim.x - 1) {
        a.ticket[0] = 0;
        if (a.step) a.step[0] += 1;
      }
    }
  } else if (i == 0 && a.step) {
    a.step[0] += 1;
  }
  if (i == 0) {
    if (a.cursor) a.cursor[0] += 1;
    if (a.rng_offset) a.rng_offset[0] += 1;
  }
}

// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int64_t lenet_wimg_elems() { return I_END; }
int64_t lenet_param_count() { return NP; }
int64_t lenet_conv_param_count() { return CNP_PAD; }
int64_t lenet_vec_len() { return VEC; }

hipError_t launch_lenet_train(const LenetTrainArgs& a, hipStream_t s) {
  if (a.B <= 0 || a.grid <= 0 || a.grid > a.B) return hipErrorInvalidValue;
  const size_t lds = (size_t)S_TOTAL;
  CSED_DISPATCH_MFMA(a.mfma_dtype, {
    hipFuncSetAttribute((const void*)lenet_train_kernel<scalar_t, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lenet_train_kernel<scalar_t, true>), dim3(a.grid), dim3(NT), lds, s, a, 0,
                       (float*)nullptr);
  });
  return hipGetLastError();
}

hipError_t launch_lenet_update(const LenetUpdateArgs& a, float* loss_parts, int nparts, float* loss_acc,
                               hipStream_t s) {
  if (a.apply_sgd && a.grad_in) {
    CSED_DISPATCH_MFMA(a.mfma_dtype, {
      hipLaunchKernelGGL(lenet_sgd_kernel<scalar_t>, dim3(cdiv(NP, 256)), dim3(256), 0, s, a);
    });
    return hipGetLastError();
  }
  if (!a.vslab || a.B <= 0) return hipErrorInvalidValue;
  CSED_DISPATCH_MFMA(a.mfma_dtype, {
    hipLaunchKernelGGL(lenet_update_kernel<scalar_t>, dim3(NB_UPDATE), dim3(UP_NT), 0, s, a, a.vslab, a.B,
                       loss_parts, nparts, loss_acc);
  });
  return hipGetLastError();
}

hipError_t launch_lenet_pack(const float* params, uint16_t* wimg, int mfma_dtype, hipStream_t s) {
  CSED_DISPATCH_MFMA(mfma_dtype, {
    hipLaunchKernelGGL(lenet_pack_kernel<scalar_t>, dim3(cdiv(NP, 256)), dim3(256), 0, s, params,
                       (unsigned short*)wimg);
  });
  return hipGetLastError();
}

hipError_t launch_lenet_eval(const uint8_t* images, const int64_t* labels, const int64_t* order,
                             int64_t n, const uint16_t* wimg, const float* params, float mean,
                             float std_, float* out, float* logp_out, int mfma_dtype, hipStream_t s) {
  // Evaluation reuses the training kernel's forward (TRAIN = false): every
  // workgroup walks samples g, g+G, ... and writes its [loss, correct] pair
  // into `out` (2*G floats); the caller reduces them in a fixed order.
  if (n <= 0) return hipSuccess;
  LenetTrainArgs a{};
  a.images = images; a.labels = labels; a.perm = order; a.cursor = nullptr;
  a.B = (int)n; a.wimg = wimg; a.params = params; a.slab = nullptr; a.loss_acc = out;
  a.grad_scale = 0.f; a.mean = mean; a.std_ = std_; a.drop_p = 0.f; a.seed = 0; a.rng_offset = nullptr;
  a.grid = (int)std::min<int64_t>(n, 256); a.mfma_dtype = mfma_dtype;
  const size_t lds = (size_t)S_TOTAL;
  CSED_DISPATCH_MFMA(mfma_dtype, {
    hipFuncSetAttribute((const void*)lenet_train_kernel<scalar_t, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lenet_train_kernel<scalar_t, false>), dim3(a.grid), dim3(NT), lds, s, a,
                       logp_out ? 1 : 0, logp_out);
  });
  return hipGetLastError();
}

}  // namespace csed
