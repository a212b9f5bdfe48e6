// dls_loss.hip — the step after the rasterizer for gfx950.
//
// One pass over the rendered and target images computes
//   loss = w_l1 * mean|p - t| + w_mse * mean (p - t)^2          (loss_mse.py:33-44 for the
//          MSE term; the L1 term stands in for LPIPS, whose VGG weights are not available)
//   dL/dp = (w_l1 * sign(p - t) + 2 w_mse (p - t)) / n           (optional, same pass)
//   psnr_i = -10 log10(mean_i (clip(p) - clip(t))^2)             (metrics.py:12-19, per image)
// Partial sums go to a per-block array and a second one-workgroup kernel folds them in a
// fixed order (deterministic; no same-address atomics from every block).

#include "dsplat_common.h"

namespace {

constexpr int NT = 256;
constexpr int kPer = 2048;  // elements per block (8 per thread): grid = ceil(n_img / kPer) x images

__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = dsplat::wave_sum(v);
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int k = 0; k < NT / 64; ++k) s += red[k];
  __syncthreads();
  return s;  // valid in thread 0
}

// grid = (blocks per image, images). part[(img * bpi + b) * 3 + {0,1,2}] = (sum|d|, sum d^2,
// sum (clip(p) - clip(t))^2) of the block's elements.
__global__ __launch_bounds__(NT) void k_loss_partial(int64_t n_img, const float* __restrict__ pred,
                                                     const float* __restrict__ tgt, float gscale_l1,
                                                     float gscale_mse, float* __restrict__ grad,
                                                     float* __restrict__ part) {
  __shared__ float red[NT / 64];
  const int img = blockIdx.y;
  const int64_t base = (int64_t)img * n_img + (int64_t)blockIdx.x * kPer;
  const int64_t end = min((int64_t)(blockIdx.x + 1) * kPer, n_img) + (int64_t)img * n_img;
  float a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int64_t i = base + threadIdx.x; i < end; i += NT) {
    const float p = pred[i], t = tgt[i];
    const float d = p - t;
    a1 += fabsf(d);
    a2 += d * d;
    const float dc = fminf(fmaxf(p, 0.f), 1.f) - fminf(fmaxf(t, 0.f), 1.f);
    a3 += dc * dc;
    if (grad) grad[i] = gscale_l1 * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) + gscale_mse * 2.f * d;
  }
  const float s1 = block_sum(a1, red), s2 = block_sum(a2, red), s3 = block_sum(a3, red);
  if (threadIdx.x == 0) {
    float* o = part + ((size_t)img * gridDim.x + blockIdx.x) * 3;
    o[0] = s1;
    o[1] = s2;
    o[2] = s3;
  }
}

// one workgroup: fixed-order fold of the partials -> loss[0] (and psnr per image)
__global__ __launch_bounds__(NT) void k_loss_final(int n_images, int bpi, int64_t n_img, float w_l1, float w_mse,
                                                   const float* __restrict__ part, float* __restrict__ loss,
                                                   float* __restrict__ psnr) {
  __shared__ float red[NT / 64];
  float a1 = 0.f, a2 = 0.f;
  for (int k = threadIdx.x; k < n_images * bpi; k += NT) {
    a1 += part[3 * k];
    a2 += part[3 * k + 1];
  }
  const float s1 = block_sum(a1, red), s2 = block_sum(a2, red);
  const double n = (double)n_img * n_images;
  if (threadIdx.x == 0) loss[0] = (float)(w_l1 * (double)s1 / n + w_mse * (double)s2 / n);
  if (psnr)
    for (int img = threadIdx.x; img < n_images; img += NT) {
      float s = 0.f;
      for (int b = 0; b < bpi; ++b) s += part[((size_t)img * bpi + b) * 3 + 2];
      psnr[img] = -10.f * log10f(s / (float)n_img);
    }
}

}  // namespace

extern "C" {

size_t dls_loss_workspace_size(int n_images, int64_t n_per_image) {
  const int64_t bpi = (n_per_image + kPer - 1) / kPer;
  return (size_t)n_images * (size_t)bpi * 3 * sizeof(float);
}

int dls_l1_mse_psnr(int n_images, int64_t n_per_image, const float* pred, const float* target, float w_l1,
                    float w_mse, float* loss, float* grad, float* psnr, void* workspace, void* stream) {
  DSPLAT_REQUIRE(n_images > 0 && n_per_image > 0, "dls_l1_mse_psnr: bad sizes");
  DSPLAT_REQUIRE(pred && target && loss && workspace, "dls_l1_mse_psnr: null pointer");
  const int64_t bpi = (n_per_image + kPer - 1) / kPer;
  DSPLAT_REQUIRE(bpi < (1 << 30) && n_images < 65536, "dls_l1_mse_psnr: too large");
  hipStream_t st = (hipStream_t)stream;
  const double n = (double)n_per_image * n_images;
  float* part = static_cast<float*>(workspace);
  dim3 grid((unsigned)bpi, (unsigned)n_images);
  k_loss_partial<<<grid, NT, 0, st>>>(n_per_image, pred, target, (float)(w_l1 / n), (float)(w_mse / n), grad, part);
  if (int e = dsplat::check_launch("k_loss_partial")) return e;
  k_loss_final<<<1, NT, 0, st>>>(n_images, (int)bpi, n_per_image, w_l1, w_mse, part, loss, psnr);
  return dsplat::check_launch("k_loss_final");
}

}  // extern "C"
