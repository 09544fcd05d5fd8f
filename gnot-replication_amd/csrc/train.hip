// The training step on either side of the GNOT path, on the GPU:
//
//   rel_l2_*  RelL2Loss (reference loss.py:14-23) over packed predictions: per-sample segment sums
//             of (p - t)^2 and t^2 (the dgl SumPooling of loss.py:20-21), loss = mean over (sample,
//             channel) of sqrt(num / den), and d loss / d pred in the same pass.  Deterministic:
//             per-split partial sums reduced in a fixed order, no atomics.
//   adamw     torch.optim.AdamW's update (main.py:51; decoupled weight decay, bias-corrected moments)
//             over ONE flat fp32 arena of parameters / gradients / moments, in torch's op order.
//             Hyper-parameters come from a small device array so a captured hipGraph replays
//             whatever the host's schedule (OneCycleLR, main.py:52/106) wrote there.
#include "gnot_common.h"
#include "gnot_kernels.h"

namespace gnot {

constexpr int kLossRows = 2048;   // rows per partial-sum workgroup

// partial[b][split][0..2C) = (sum (p-t)^2 [C], sum t^2 [C]) over the split's rows of sample b
__global__ void __launch_bounds__(256) rel_l2_partial_kernel(const float* __restrict__ pred,
                                                             const float* __restrict__ tgt,
                                                             const long* __restrict__ off, int C, int nsplit,
                                                             float* __restrict__ partial) {
  __shared__ float red[256 * 2];
  const int b = blockIdx.x / nsplit, split = blockIdx.x % nsplit;
  const long r0 = off[b] + (long)split * kLossRows;
  const long r1 = min(off[b + 1], r0 + kLossRows);
  for (int c = 0; c < C; ++c) {
    float num = 0.f, den = 0.f;
    for (long r = r0 + threadIdx.x; r < r1; r += 256) {
      const float t = tgt[r * C + c];
      const float d = pred[r * C + c] - t;
      num = fmaf(d, d, num);
      den = fmaf(t, t, den);
    }
    red[threadIdx.x] = num;
    red[256 + threadIdx.x] = den;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (threadIdx.x < s) {
        red[threadIdx.x] += red[threadIdx.x + s];
        red[256 + threadIdx.x] += red[256 + threadIdx.x + s];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      float* P = partial + ((long)b * nsplit + split) * 2 * C;
      P[c] = red[0];
      P[C + c] = red[256];
    }
    __syncthreads();
  }
}

// one workgroup: num/den per (b, c) in split order, loss = mean sqrt(num/den), and the per-(b, c)
// gradient scale d loss / d pred = (p - t) / (B C den sqrt(num/den))
__global__ void __launch_bounds__(256) rel_l2_finish_kernel(const float* __restrict__ partial, int B, int C,
                                                            int nsplit, float* __restrict__ scale,
                                                            float* __restrict__ loss) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int i = threadIdx.x; i < B * C; i += 256) {
    const int b = i / C, c = i % C;
    float num = 0.f, den = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      const float* P = partial + ((long)b * nsplit + s) * 2 * C;
      num += P[c];
      den += P[C + c];
    }
    const float r = sqrtf(num / den);
    acc += r;
    scale[i] = 1.0f / ((float)(B * C) * den * r);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0] / (float)(B * C);
}

__global__ void __launch_bounds__(256) rel_l2_grad_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                                          const long* __restrict__ off, int B, int C,
                                                          const float* __restrict__ scale, float* __restrict__ dpred,
                                                          long rows) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * C) return;
  const long r = i / C;
  const int c = (int)(i % C);
  int lo = 0, hi = B - 1;                           // sample of row r
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= r) lo = mid; else hi = mid - 1;
  }
  dpred[i] = (pred[i] - tgt[i]) * scale[lo * C + c];
}

int rel_l2_splits(const long* off_host, int B) {
  long mx = 1;
  for (int b = 0; b < B; ++b) mx = std::max(mx, off_host[b + 1] - off_host[b]);
  return (int)((mx + kLossRows - 1) / kLossRows);
}

hipError_t launch_rel_l2(const float* pred, const float* tgt, const long* off_dev, int B, int C, int nsplit,
                         long rows, float* work, float* loss, float* dpred, hipStream_t s) {
  float* partial = work;                                  // [B][nsplit][2C]
  float* scale = work + (size_t)B * nsplit * 2 * C;       // [B][C]
  hipLaunchKernelGGL(rel_l2_partial_kernel, dim3(B * nsplit), dim3(256), 0, s, pred, tgt, off_dev, C, nsplit, partial);
  hipLaunchKernelGGL(rel_l2_finish_kernel, dim3(1), dim3(256), 0, s, (const float*)partial, B, C, nsplit, scale, loss);
  if (dpred && rows > 0)
    hipLaunchKernelGGL(rel_l2_grad_kernel, dim3((unsigned)((rows * C + 255) / 256)), dim3(256), 0, s, pred, tgt,
                       off_dev, B, C, (const float*)scale, dpred, rows);
  return hipGetLastError();
}

// ---------------------------------------------------------------- AdamW over a flat arena
// hyper = {lr, beta1, beta2, eps, weight_decay, bias_correction1, bias_correction2, grad_scale}
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                    float* __restrict__ m, float* __restrict__ v, long n,
                                                    const float* __restrict__ hyper) {
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float bc1 = hyper[5], bc2 = hyper[6], gs = hyper[7];
  const float step_size = lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float g = grad[i] * gs;
    float p = param[i] * (1.0f - lr * wd);              // decoupled weight decay
    float mi = m[i];
    mi = mi + (1.0f - b1) * (g - mi);                   // exp_avg.lerp_(grad, 1 - beta1)
    const float vi = v[i] * b2 + (1.0f - b2) * g * g;   // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p = p - step_size * (mi / denom);                   // param.addcdiv_(exp_avg, denom, -step_size)
    param[i] = p;
    m[i] = mi;
    v[i] = vi;
  }
}

hipError_t launch_adamw(float* param, const float* grad, float* m, float* v, long n, const float* hyper,
                        hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const long blocks = std::min<long>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, s, param, grad, m, v, n, hyper);
  return hipGetLastError();
}

}  // namespace gnot
