// Small memory-bound kernels: data gather+normalise, flat SGD, log-softmax,
// NLL, max-pool+ReLU, dropout and the ReLU/dropout gate backward.
//
// Parity targets (reference behaviour, re-implemented natively):
//   gather_normalize  <- torchvision ToTensor+Normalize((0.1307,),(0.3081,))
//                        + DataLoader collation   (ref src/train_dist.py:16-19,40-45)
//   sgd_flat          <- torch.optim.SGD(lr, momentum)      (ref src/train.py:60-61)
//   log_softmax / nll <- F.log_softmax(dim=1), F.nll_loss   (ref src/model.py:22, src/train.py:74)
//   maxpool_relu      <- F.relu(F.max_pool2d(x, 2))         (ref src/model.py:16-17)
//   dropout           <- F.dropout / nn.Dropout2d           (ref src/model.py:11,17,20)
#include "common.h"
#include "dispatch.h"

namespace csed {

// ---------------------------------------------------------------------------
// Data: batch gather + normalise.  One block per sample row, 16-byte loads.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void gather_normalize_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ idx,
                                        const int64_t* __restrict__ cursor, int B, int elems,
                                        float mean, float inv_std, T* __restrict__ out,
                                        int64_t* __restrict__ labels_out,
                                        const int64_t* __restrict__ labels_src) {
  const int b = blockIdx.x;
  const int64_t base = cursor ? cursor[0] * (int64_t)B : 0;
  const int64_t row = idx[base + b];
  const uint8_t* s = src + row * (int64_t)elems;
  T* o = out + (int64_t)b * elems;
  const float scale = inv_std * (1.0f / 255.0f);
  const float shift = -mean * inv_std;
  for (int i = threadIdx.x; i < elems; i += blockDim.x) o[i] = from_f32<T>(fmaf((float)s[i], scale, shift));
  if (labels_out && threadIdx.x == 0) labels_out[b] = labels_src[row];
}

hipError_t launch_gather_normalize(const uint8_t* src, const int64_t* idx, const int64_t* cursor,
                                   int64_t n_src, int B, int elems, float mean, float std_,
                                   void* out, int out_dtype, int64_t* labels_out,
                                   const int64_t* labels_src, hipStream_t s) {
  (void)n_src;
  if (B <= 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(out_dtype, {
    hipLaunchKernelGGL(gather_normalize_kernel<scalar_t>, dim3(B), dim3(256), 0, s, src, idx, cursor,
                       B, elems, mean, 1.0f / std_, (scalar_t*)out, labels_out, labels_src);
  });
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// SGD with momentum, torch.optim.SGD semantics:
//   g' = g*scale + wd*p
//   buf = (step==0) ? g' : m*buf + (1-dampening)*g'
//   d = nesterov ? g' + m*buf : buf ;  p -= lr*d
// The last block to finish bumps step[0] (ticket protocol; every block has
// read step[0] before it takes its ticket).
// ---------------------------------------------------------------------------
__global__ void sgd_flat_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                                int64_t n, float lr, float m, float damp, float wd, int nesterov,
                                float gscale, int64_t* step, int* ticket) {
  const bool first = step[0] == 0;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 bv = first ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<float4*>(buf)[i];
    float* pp = &pv.x; float* gg = &gv.x; float* bb = &bv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gg[j] * gscale + wd * pp[j];
      float bj = (m != 0.f) ? (first ? gj : fmaf(m, bb[j], (1.f - damp) * gj)) : gj;
      float d = (m != 0.f) ? (nesterov ? fmaf(m, bj, gj) : bj) : gj;
      bb[j] = bj;
      pp[j] = fmaf(-lr, d, pp[j]);
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    if (m != 0.f) reinterpret_cast<float4*>(buf)[i] = bv;
  }
  // scalar tail
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float gj = g[i] * gscale + wd * p[i];
    float bj = (m != 0.f) ? (first ? gj : fmaf(m, buf[i], (1.f - damp) * gj)) : gj;
    float d = (m != 0.f) ? (nesterov ? fmaf(m, bj, gj) : bj) : gj;
    if (m != 0.f) buf[i] = bj;
    p[i] = fmaf(-lr, d, p[i]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = atomicAdd(ticket, 1);
    if (t == (int)gridDim.x - 1) {
      ticket[0] = 0;
      step[0] = step[0] + 1;
    }
  }
}

hipError_t launch_sgd_flat(float* p, const float* g, float* buf, int64_t n, float lr, float momentum,
                           float dampening, float weight_decay, int nesterov, float grad_scale,
                           int64_t* step, int* ticket, hipStream_t s) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)buf) & 15) return hipErrorInvalidValue;
  int blocks = (int)std::min<int64_t>(std::max<int64_t>(cdiv(n / 4 + 1, 256), 1), 1024);
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(blocks), dim3(256), 0, s, p, g, buf, n, lr, momentum,
                     dampening, weight_decay, nesterov, grad_scale, step, ticket);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// log_softmax (one wave per row) / backward / NLL
// ---------------------------------------------------------------------------
template <typename T>
__global__ void log_softmax_fwd_kernel(const T* __restrict__ x, float* __restrict__ y, int rows, int C) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + wave;
  if (r >= rows) return;
  const T* xr = x + (int64_t)r * C;
  float mx = -INFINITY;
  for (int c = lane; c < C; c += 64) mx = fmaxf(mx, to_f32(xr[c]));
  mx = wave_max(mx);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(to_f32(xr[c]) - mx);
  s = wave_sum(s);
  const float lse = mx + __logf(s);
  for (int c = lane; c < C; c += 64) y[(int64_t)r * C + c] = to_f32(xr[c]) - lse;
}

hipError_t launch_log_softmax_fwd(const void* x, int x_dtype, float* y, int rows, int C, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(x_dtype, {
    hipLaunchKernelGGL(log_softmax_fwd_kernel<scalar_t>, dim3(cdiv(rows, 4)), dim3(256), 0, s,
                       (const scalar_t*)x, y, rows, C);
  });
  return hipGetLastError();
}

template <typename T>
__global__ void log_softmax_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                       T* __restrict__ dx, int rows, int C) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x >> 6) + wave;
  if (r >= rows) return;
  const int64_t o = (int64_t)r * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += dy[o + c];
  s = wave_sum(s);
  for (int c = lane; c < C; c += 64) dx[o + c] = from_f32<T>(dy[o + c] - __expf(y[o + c]) * s);
}

hipError_t launch_log_softmax_bwd(const float* dy, const float* y, void* dx, int dx_dtype, int rows,
                                  int C, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(dx_dtype, {
    hipLaunchKernelGGL(log_softmax_bwd_kernel<scalar_t>, dim3(cdiv(rows, 4)), dim3(256), 0, s, dy, y,
                       (scalar_t*)dx, rows, C);
  });
  return hipGetLastError();
}

// Single-block NLL so the mean/sum reduction is in a fixed order (bitwise
// reproducible).  Rows are strided over the block's threads, then reduced.
__global__ void nll_fwd_kernel(const float* __restrict__ logp, const int64_t* __restrict__ target,
                               float* __restrict__ out, int rows, int C, int reduction,
                               int64_t* __restrict__ correct) {
  __shared__ float ssum[256];
  __shared__ int scor[256];
  float acc = 0.f;
  int cor = 0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    const int64_t t = target[r];
    const float v = -logp[(int64_t)r * C + t];
    if (reduction == 0) out[r] = v;
    acc += v;
    if (correct) {
      int best = 0;
      float bv = logp[(int64_t)r * C];
      for (int c = 1; c < C; ++c) {
        float q = logp[(int64_t)r * C + c];
        if (q > bv) { bv = q; best = c; }
      }
      cor += (best == t);
    }
  }
  ssum[threadIdx.x] = acc;
  scor[threadIdx.x] = cor;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      ssum[threadIdx.x] += ssum[threadIdx.x + o];
      scor[threadIdx.x] += scor[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (reduction == 1) out[0] = ssum[0] / (float)rows;
    else if (reduction == 2) out[0] = ssum[0];
    if (correct) correct[0] = scor[0];
  }
}

hipError_t launch_nll_fwd(const float* logp, const int64_t* target, float* out, int rows, int C,
                          int reduction, int64_t* correct, hipStream_t s) {
  hipLaunchKernelGGL(nll_fwd_kernel, dim3(1), dim3(256), 0, s, logp, target, out, rows, C, reduction,
                     correct);
  return hipGetLastError();
}

__global__ void nll_bwd_kernel(const float* __restrict__ gout, const int64_t* __restrict__ target,
                               float* __restrict__ d, int rows, int C, int reduction) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  const int r = (int)(i / C), c = (int)(i % C);
  float g = reduction == 0 ? gout[r] : gout[0];
  if (reduction == 1) g /= (float)rows;
  d[i] = (c == target[r]) ? -g : 0.f;
}

hipError_t launch_nll_bwd(const float* gout, const int64_t* target, float* dlogp, int rows, int C,
                          int reduction, hipStream_t s) {
  int64_t n = (int64_t)rows * C;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(nll_bwd_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, gout, target, dlogp, rows, C,
                     reduction);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// log_softmax + NLL in one launch each way (the modular step's loss: nll(log_softmax(z)), ref
// src/model.py:22 + src/train.py:74 / train_dist.py:67,82 -- four launches as separate ops).
// Forward: one block, a thread per row (rows strided over the block), log-probs kept for the
// backward, the mean / sum reduced in a fixed order (bitwise reproducible).  Backward: one
// thread per element, dz = g_r * (exp(logp) - onehot).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) lsm_nll_fwd_kernel(const T* __restrict__ z, const int64_t* __restrict__ target,
                                                          float* __restrict__ logp, float* __restrict__ out, int rows,
                                                          int C, int reduction) {
  __shared__ float ssum[256];
  float acc = 0.f;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    const T* zr = z + (int64_t)r * C;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, to_f32(zr[c]));
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(to_f32(zr[c]) - mx);
    const float lse = mx + __logf(s);
    const int64_t t = target[r];
    float* lr = logp + (int64_t)r * C;
    float v = 0.f;
    for (int c = 0; c < C; ++c) {
      const float q = to_f32(zr[c]) - lse;
      lr[c] = q;
      if (c == t) v = -q;
    }
    if (reduction == 0) out[r] = v;
    acc += v;
  }
  ssum[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) ssum[threadIdx.x] += ssum[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (reduction == 1) out[0] = ssum[0] / (float)rows;
    else if (reduction == 2) out[0] = ssum[0];
  }
}

hipError_t launch_lsm_nll_fwd(const void* z, int z_dtype, const int64_t* target, float* logp, float* out, int rows,
                              int C, int reduction, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(z_dtype, {
    hipLaunchKernelGGL(lsm_nll_fwd_kernel<scalar_t>, dim3(1), dim3(256), 0, s, (const scalar_t*)z, target, logp,
                       out, rows, C, reduction);
  });
  return hipGetLastError();
}

template <typename T>
__global__ void lsm_nll_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ logp,
                                   const int64_t* __restrict__ target, T* __restrict__ dz, int rows, int C,
                                   int reduction) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  const int r = (int)(i / C), c = (int)(i - (int64_t)r * C);
  float g = reduction == 0 ? gout[r] : gout[0];
  if (reduction == 1) g /= (float)rows;
  dz[i] = from_f32<T>(g * (__expf(logp[i]) - (c == target[r] ? 1.f : 0.f)));
}

hipError_t launch_lsm_nll_bwd(const float* gout, const float* logp, const int64_t* target, void* dz, int dz_dtype,
                              int rows, int C, int reduction, hipStream_t s) {
  const int64_t n = (int64_t)rows * C;
  if (n == 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(dz_dtype, {
    hipLaunchKernelGGL(lsm_nll_bwd_kernel<scalar_t>, dim3(cdiv(n, 256)), dim3(256), 0, s, gout, logp, target,
                       (scalar_t*)dz, rows, C, reduction);
  });
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// max-pool (k x k, stride k) + ReLU (+ per-channel scale) forward / backward
// One thread per pooled output.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void maxpool_relu_fwd_kernel(const T* __restrict__ x, T* __restrict__ out, uint8_t* __restrict__ idx,
                                        const float* __restrict__ chscale, int N, int C, int H, int W, int k) {
  const int PH = H / k, PW = W / k;
  const int64_t total = (int64_t)N * C * PH * PW;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int pw = (int)(i % PW);
  const int ph = (int)((i / PW) % PH);
  const int64_t nc = i / ((int64_t)PH * PW);
  const T* xp = x + nc * H * W + (int64_t)(ph * k) * W + pw * k;
  float best = to_f32(xp[0]);
  int bi = 0;
  for (int dy = 0; dy < k; ++dy)
    for (int dx = 0; dx < k; ++dx) {
      float v = to_f32(xp[dy * W + dx]);
      if (v > best || (v != v)) { best = v; bi = dy * k + dx; }  // NaN propagates like torch
    }
  float sc = chscale ? chscale[nc] : 1.f;
  float o = (best > 0.f ? best : (best != best ? best : 0.f)) * sc;
  out[i] = from_f32<T>(o);
  idx[i] = (uint8_t)bi;
}

hipError_t launch_maxpool_relu_fwd(const void* x, int dtype, void* out, uint8_t* idx,
                                   const float* chscale, int N, int C, int H, int W, int k,
                                   hipStream_t s) {
  int64_t total = (int64_t)N * C * (H / k) * (W / k);
  if (total == 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(dtype, {
    hipLaunchKernelGGL(maxpool_relu_fwd_kernel<scalar_t>, dim3(cdiv(total, 256)), dim3(256), 0, s,
                       (const scalar_t*)x, (scalar_t*)out, idx, chscale, N, C, H, W, k);
  });
  return hipGetLastError();
}

template <typename TD, typename TO, typename TX>
__global__ void maxpool_relu_bwd_kernel(const TD* __restrict__ dout, const TO* __restrict__ out,
                                        const uint8_t* __restrict__ idx, const float* __restrict__ chscale,
                                        TX* __restrict__ dx, int N, int C, int H, int W, int k) {
  // one thread per INPUT element so every dx element is written exactly once
  const int64_t total = (int64_t)N * C * H * W;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int w = (int)(i % W);
  const int h = (int)((i / W) % H);
  const int64_t nc = i / ((int64_t)H * W);
  const int PH = H / k, PW = W / k;
  const int ph = h / k, pw = w / k;
  float g = 0.f;
  if (ph < PH && pw < PW) {
    const int64_t o = nc * PH * PW + (int64_t)ph * PW + pw;
    if ((int)idx[o] == (h - ph * k) * k + (w - pw * k) && to_f32(out[o]) > 0.f)
      g = to_f32(dout[o]) * (chscale ? chscale[nc] : 1.f);
  }
  dx[i] = from_f32<TX>(g);
}

// 2x2 windows with even H, W: one thread per POOLED element writing its window's four dx values
// (the one-thread-per-input-element form above does three 64-bit divisions per element: 22 us for
// the modular step's [4096, 20, 8, 8] conv2 gradient, profiles/r6/modular).  A block takes whole
// (n, c) planes, so the index math is 32-bit divisions by the block-uniform plane size.
template <typename TD, typename TX>
__global__ void maxpool2_relu_bwd_kernel(const TD* __restrict__ dout, const TX* __restrict__ out,
                                         const uint8_t* __restrict__ idx, const float* __restrict__ chscale,
                                         TX* __restrict__ dx, int planes, int PH, int PW) {
  const int per = PH * PW;
  const int ppb = max(1, (int)blockDim.x / per);  // planes per block
  for (int t = threadIdx.x; t < ppb * per; t += blockDim.x) {
    const int q = t / per;
    const int pl = blockIdx.x * ppb + q;
    if (pl >= planes) break;
    const int r = t - q * per, ph = r / PW, pw = r - ph * PW;
    const int64_t o = (int64_t)pl * per + r;
    const int sel = idx[o];
    const float g = to_f32(out[o]) > 0.f ? to_f32(dout[o]) * (chscale ? chscale[pl] : 1.f) : 0.f;
    TX* d = dx + (int64_t)pl * 4 * per + (2 * ph) * (2 * PW) + 2 * pw;
    d[0] = from_f32<TX>(sel == 0 ? g : 0.f);
    d[1] = from_f32<TX>(sel == 1 ? g : 0.f);
    d[2 * PW] = from_f32<TX>(sel == 2 ? g : 0.f);
    d[2 * PW + 1] = from_f32<TX>(sel == 3 ? g : 0.f);
  }
}

hipError_t launch_maxpool_relu_bwd(const void* dout, int dout_dtype, const void* out, int out_dtype,
                                   const uint8_t* idx, const float* chscale, void* dx, int dx_dtype,
                                   int N, int C, int H, int W, int k, hipStream_t s) {
  int64_t total = (int64_t)N * C * H * W;
  if (total == 0) return hipSuccess;
  if (out_dtype != dx_dtype) return hipErrorInvalidValue;
  if (k == 2 && !(H & 1) && !(W & 1) && (int64_t)N * C < INT32_MAX) {
    const int planes = N * C, PH = H / 2, PW = W / 2, ppb = std::max(1, 256 / (PH * PW));
    const dim3 grid(cdiv(planes, ppb));
    CSED_DISPATCH_FLOAT(dx_dtype, {
      typedef scalar_t TX;
      if (dout_dtype == kF32) {
        hipLaunchKernelGGL((maxpool2_relu_bwd_kernel<float, TX>), grid, dim3(256), 0, s, (const float*)dout,
                           (const TX*)out, idx, chscale, (TX*)dx, planes, PH, PW);
      } else if (dout_dtype == dx_dtype) {
        hipLaunchKernelGGL((maxpool2_relu_bwd_kernel<TX, TX>), grid, dim3(256), 0, s, (const TX*)dout,
                           (const TX*)out, idx, chscale, (TX*)dx, planes, PH, PW);
      } else {
        return hipErrorInvalidValue;
      }
    });
    return hipGetLastError();
  }
  CSED_DISPATCH_FLOAT(dx_dtype, {
    typedef scalar_t TX;
    if (dout_dtype == kF32) {
      hipLaunchKernelGGL((maxpool_relu_bwd_kernel<float, TX, TX>), dim3(cdiv(total, 256)), dim3(256), 0, s,
                         (const float*)dout, (const TX*)out, idx, chscale, (TX*)dx, N, C, H, W, k);
    } else if (dout_dtype == dx_dtype) {
      hipLaunchKernelGGL((maxpool_relu_bwd_kernel<TX, TX, TX>), dim3(cdiv(total, 256)), dim3(256), 0, s,
                         (const TX*)dout, (const TX*)out, idx, chscale, (TX*)dx, N, C, H, W, k);
    } else {
      return hipErrorInvalidValue;
    }
  });
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Dropout
// ---------------------------------------------------------------------------
template <typename T>
__global__ void dropout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t total, int64_t inner,
                                   int channel_mode, float p, uint64_t seed, uint64_t offset,
                                   const int64_t* __restrict__ offset_dev) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint64_t off = rng_offset(offset, offset_dev);
  const int64_t e = channel_mode ? i / inner : i;
  const bool keep = dropout_keep(seed, off, (uint64_t)e, p);
  const float sc = p < 1.f ? 1.f / (1.f - p) : 0.f;
  y[i] = from_f32<T>(keep ? to_f32(x[i]) * sc : 0.f);
}

hipError_t launch_dropout_fwd(const void* x, int dtype, void* y, int64_t rows, int64_t C,
                              int64_t inner, int channel_mode, float p, uint64_t seed,
                              uint64_t offset, const int64_t* offset_dev, hipStream_t s) {
  int64_t total = rows * C * inner;
  if (total == 0) return hipSuccess;
  CSED_DISPATCH_FLOAT(dtype, {
    hipLaunchKernelGGL(dropout_fwd_kernel<scalar_t>, dim3(cdiv(total, 256)), dim3(256), 0, s,
                       (const scalar_t*)x, (scalar_t*)y, total, inner, channel_mode, p, seed, offset,
                       offset_dev);
  });
  return hipGetLastError();
}

__global__ void channel_mask_kernel(float* __restrict__ sc, int64_t n, float p, uint64_t seed, uint64_t offset,
                                    const int64_t* __restrict__ offset_dev) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = rng_offset(offset, offset_dev);
  sc[i] = dropout_keep(seed, off, (uint64_t)i, p) ? (p < 1.f ? 1.f / (1.f - p) : 0.f) : 0.f;
}

hipError_t launch_channel_mask(float* scale, int64_t n, float p, uint64_t seed, uint64_t offset,
                               const int64_t* offset_dev, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(channel_mask_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, scale, n, p, seed, offset,
                     offset_dev);
  return hipGetLastError();
}

template <typename TD, typename TY, typename TX>
__global__ void gate_bwd_kernel(const TD* __restrict__ dout, const TY* __restrict__ y, TX* __restrict__ dx,
                                int64_t n, float s) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  dx[i] = from_f32<TX>(to_f32(y[i]) > 0.f ? to_f32(dout[i]) * s : 0.f);
}

hipError_t launch_gate_bwd(const void* dout, int dout_dtype, const void* y, int y_dtype, void* dx,
                           int dx_dtype, int64_t n, float s, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (dout_dtype != dx_dtype) return hipErrorInvalidValue;
  CSED_DISPATCH_FLOAT(dx_dtype, {
    typedef scalar_t TX;
    switch (y_dtype) {
      case kF32:
        hipLaunchKernelGGL((gate_bwd_kernel<TX, float, TX>), dim3(cdiv(n, 256)), dim3(256), 0, st,
                           (const TX*)dout, (const float*)y, (TX*)dx, n, s);
        break;
      case kBF16:
        hipLaunchKernelGGL((gate_bwd_kernel<TX, __bf16, TX>), dim3(cdiv(n, 256)), dim3(256), 0, st,
                           (const TX*)dout, (const __bf16*)y, (TX*)dx, n, s);
        break;
      case kF16:
        hipLaunchKernelGGL((gate_bwd_kernel<TX, _Float16, TX>), dim3(cdiv(n, 256)), dim3(256), 0, st,
                           (const TX*)dout, (const _Float16*)y, (TX*)dx, n, s);
        break;
      default: return hipErrorInvalidValue;
    }
  });
  return hipGetLastError();
}

// Load this translation unit's code object on the current device now (the HIP runtime loads it
// lazily, at the TU's first launch): csed::preload_kernels, so a cold epoch does not pay it.
hipError_t preload_elementwise() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(sgd_flat_kernel));
}

}  // namespace csed
