// dga_math.h — the Gaussian adapter's per-row math (encoder glue + GaussianAdapter + rotate_sh),
// shared by dga_adapter.hip (k_adapter_fwd / k_adapter_bwd) and the fused head backward in
// dsr_raster.hip (k_head_bwd), so both evaluate exactly the same float operations.
#pragma once
#include "dsplat_common.h"

namespace dga {

constexpr float kC0 = 0.28209479177387814f;
constexpr int kCamFloats = 104;  // R[9] t[3] Kinv[9] D1[9] D2[25] D3[49]
constexpr int kOffR = 0, kOffT = 9, kOffKinv = 12, kOffD1 = 21, kOffD2 = 30, kOffD3 = 55;

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + __expf(-x)); }

// torch.nn.functional.softplus (beta 1, threshold 20)
__device__ __forceinline__ float softplusf(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float softplus_grad(float x) { return x > 20.0f ? 1.0f : 1.0f / (1.0f + expf(-x)); }

struct QuatR {
  float R[9];
  float s2;  // 2 / (|q|^2 + eps)
};

// quaternion_to_matrix (gaussians.py:8-30), q = (i, j, k, r)
__device__ __forceinline__ void quat_to_R(const float q[4], QuatR& o) {
  const float i = q[0], j = q[1], k = q[2], r = q[3];
  const float n = ((i * i + j * j) + k * k) + r * r;
  const float s = 2.0f / (n + 1e-8f);
  o.s2 = s;
  o.R[0] = 1.0f - s * (j * j + k * k);
  o.R[1] = s * (i * j - k * r);
  o.R[2] = s * (i * k + j * r);
  o.R[3] = s * (i * j + k * r);
  o.R[4] = 1.0f - s * (i * i + k * k);
  o.R[5] = s * (j * k - i * r);
  o.R[6] = s * (i * k - j * r);
  o.R[7] = s * (j * k + i * r);
  o.R[8] = 1.0f - s * (i * i + j * j);
}

// C = A B (3x3 row-major), sums in k order
__device__ __forceinline__ void mm3(const float* A, const float* B, float* C) {
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c) C[a * 3 + c] = (A[a * 3] * B[c] + A[a * 3 + 1] * B[3 + c]) + A[a * 3 + 2] * B[6 + c];
}
// C = A B^T
__device__ __forceinline__ void mm3t(const float* A, const float* B, float* C) {
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[a * 3 + c] = (A[a * 3] * B[c * 3] + A[a * 3 + 1] * B[c * 3 + 1]) + A[a * 3 + 2] * B[c * 3 + 2];
}
// C = A^T B
__device__ __forceinline__ void mmt3(const float* A, const float* B, float* C) {
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c) C[a * 3 + c] = (A[a] * B[c] + A[3 + a] * B[3 + c]) + A[6 + a] * B[6 + c];
}

// One launch's inputs. GLUE (the encoder glue fused in, dga_adapter_fwd): rows are head
// channels [opacity logit, 2 offset logits, raw...] per (b, v, pixel). Otherwise (the
// reference GaussianAdapter.forward signature, dga_adapter_forward): rows are the adapter's
// raw_gaussians [scales 3, rotation 4, sh 3 d_sh] and the normalised coordinates come in
// `coords` [N, 2]; S rows share one pixel (surfaces x Gaussians per pixel, innermost).
struct AdIn {
  const float* rows;    // [N, C]
  const float* coords;  // [N, 2] (reference signature only)
  const float* depths;  // [N]
  const float* images;  // [B*V, 3, H, W]
  const float* cams;    // [B*V, kCamFloats]
  const float* sh_mask; // [d_sh]
  float smin, smax, eps;
  int C, BV, H, W, S;
};

struct Pix {
  size_t n;   // row
  size_t bv;  // camera / image index
  int p, i, j;
};

__device__ __forceinline__ bool pixel_of(size_t n, const AdIn& a, Pix& px) {
  const size_t HW = (size_t)a.H * a.W, per = HW * (size_t)a.S;
  if (n >= (size_t)a.BV * per) return false;
  px.n = n;
  px.bv = n / per;
  px.p = (int)((n / (size_t)a.S) % HW);
  px.i = px.p / a.W;
  px.j = px.p - px.i * a.W;
  return true;
}

// pixel ray: x, y normalised coordinates -> u = K^-1 [x, y, 1], d = u / u.z, dw = Rc d
__device__ __forceinline__ void ray(const float* cam, float x, float y, float u[3], float d[3], float dw[3]) {
  const float* Ki = cam + kOffKinv;
#pragma unroll
  for (int a = 0; a < 3; ++a) u[a] = (Ki[a * 3] * x + Ki[a * 3 + 1] * y) + Ki[a * 3 + 2] * 1.0f;
#pragma unroll
  for (int a = 0; a < 3; ++a) d[a] = u[a] / u[2];
  const float* Rc = cam + kOffR;
#pragma unroll
  for (int a = 0; a < 3; ++a) dw[a] = (Rc[a * 3] * d[0] + Rc[a * 3 + 1] * d[1]) + Rc[a * 3 + 2] * d[2];
}

template <int NSH>
__device__ __forceinline__ const float* dblock(const float* cam, int l) {
  return cam + (l == 1 ? kOffD1 : l == 2 ? kOffD2 : kOffD3);
}

// row channels used: GLUE adds the opacity logit and the two offset logits in front
template <int NSH, bool GLUE>
struct Rows {
  static constexpr int kOff = GLUE ? 3 : 0;            // first raw_gaussians channel
  static constexpr int kHead = kOff + 7 + 3 * NSH;
};

// normalised image coordinates of a row: pixel centre + offset (GLUE) or given (reference)
template <bool GLUE>
__device__ __forceinline__ void row_xy(const AdIn& a, const Pix& px, const float* h, float& x, float& y, float& s1,
                                       float& s2) {
  if constexpr (GLUE) {
    s1 = sigmoidf(h[1]);
    s2 = sigmoidf(h[2]);
    x = ((float)px.j + 0.5f) / (float)a.W + (s1 - 0.5f) * (1.0f / (float)a.W);
    y = ((float)px.i + 0.5f) / (float)a.H + (s2 - 0.5f) * (1.0f / (float)a.H);
  } else {
    s1 = s2 = 0.f;
    x = a.coords[2 * px.n];
    y = a.coords[2 * px.n + 1];
  }
}

// The adapter's forward for one row (k_adapter_fwd's per-row math; the fused head backward
// of dsr_raster.hip re-evaluates it with the same operations, so its values are the same
// floats the forward wrote). opac: written when non-NULL (GLUE).
template <int NSH, bool GLUE>
__device__ __forceinline__ void adapter_row_fwd(const AdIn& a, const Pix& px, const float* cam, const float* h,
                                                float* __restrict__ opac, float (&mo)[3], float (&Cw)[9],
                                                float (&ho)[3 * NSH], float (&sc)[3], float (&q)[4]) {
  constexpr int O = Rows<NSH, GLUE>::kOff;
  const size_t HW = (size_t)a.H * a.W;
      if constexpr (GLUE)
    if (opac) opac[px.n] = sigmoidf(h[0]);
      // position: the camera ray through the row's image coordinates, scaled by the depth
      float x, y, s1, s2;
      row_xy<GLUE>(a, px, h, x, y, s1, s2);
      float u[3], d[3], dw[3];
      ray(cam, x, y, u, d, dw);
      const float z = a.depths[px.n];
  #pragma unroll
      for (int k = 0; k < 3; ++k) mo[k] = cam[kOffT + k] + dw[k] * z;
      // covariance
  #pragma unroll
      for (int k = 0; k < 3; ++k) sc[k] = fminf(fmaxf(softplusf(h[O + k] - 4.0f), a.smin), a.smax);
      const float L = sqrtf(((h[O + 3] * h[O + 3] + h[O + 4] * h[O + 4]) + h[O + 5] * h[O + 5]) + h[O + 6] * h[O + 6]);
  #pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = h[O + 3 + k] / (L + a.eps);
      QuatR qr;
      quat_to_R(q, qr);
      float M[9], Cl[9], T1[9];
  #pragma unroll
      for (int r = 0; r < 3; ++r)
  #pragma unroll
        for (int k = 0; k < 3; ++k) M[r * 3 + k] = (qr.R[r * 3 + k] * sc[k]) * sc[k];
      mm3t(M, qr.R, Cl);          // (R S S^T) R^T
      mm3(cam + kOffR, Cl, T1);   // Rc C
      mm3t(T1, cam + kOffR, Cw);  // (Rc C) Rc^T
      // harmonics: masked raw SH + the image colour in the DC term, rotated per degree block
  #pragma unroll
      for (int c = 0; c < 3; ++c) {
        float sh[NSH];
  #pragma unroll
        for (int k = 0; k < NSH; ++k) sh[k] = h[O + 7 + c * NSH + k] * a.sh_mask[k];
        sh[0] = sh[0] + (a.images[px.bv * 3 * HW + px.p + c * HW] - 0.5f) / kC0;
        float* o = ho + c * NSH;
        o[0] = sh[0];
  #pragma unroll
        for (int l = 1; l * l < NSH; ++l) {
          const int n = 2 * l + 1, b0 = l * l;
          const float* D = dblock<NSH>(cam, l);
  #pragma unroll
          for (int a2 = 0; a2 < n; ++a2) {
            float acc = 0.0f;
  #pragma unroll
            for (int k = 0; k < n; ++k) acc = acc + D[a2 * n + k] * sh[b0 + k];
            o[b0 + a2] = acc;
          }
        }
      }
}

// The adapter's backward for one row (k_adapter_bwd's per-row math), from the output gradients
// gm (means), gCw (covariance, full 3x3), gh (harmonics, channel-major), gop (opacity, GLUE;
// have_dopac), gsc / grot (reference signature only). dh: the row's KH channel gradients
// (zeroed by the caller); gxy: d / d image coordinates; ddepth written when non-NULL.
template <int NSH, bool GLUE>
__device__ __forceinline__ void adapter_row_bwd(const AdIn& a, const Pix& px, const float* cam, const float* h,
                                                float z, const float (&gm)[3], const float (&gCw)[9],
                                                const float (&gh)[3 * NSH], float gop, bool have_dopac,
                                                const float (&gsc)[3], const float (&grot)[4], float* dh,
                                                float (&gxy)[2], float* __restrict__ ddepth) {
  constexpr int O = Rows<NSH, GLUE>::kOff;
      if constexpr (GLUE) {  // opacity
        const float sg = sigmoidf(h[0]);
        dh[0] = have_dopac ? gop * sg * (1.0f - sg) : 0.0f;
      }
      // mean -> depth, image coordinates (-> offset logits)
      {
        float x, y, s1, s2;
        row_xy<GLUE>(a, px, h, x, y, s1, s2);
        float u[3], d[3], dw[3];
        ray(cam, x, y, u, d, dw);
        if (ddepth) ddepth[px.n] = (gm[0] * dw[0] + gm[1] * dw[1]) + gm[2] * dw[2];
        const float* Rc = cam + kOffR;
        float gd[3];  // d L / d d = Rc^T (z gm)
  #pragma unroll
        for (int k = 0; k < 3; ++k) gd[k] = (Rc[k] * gm[0] + Rc[3 + k] * gm[1]) + Rc[6 + k] * gm[2];
  #pragma unroll
        for (int k = 0; k < 3; ++k) gd[k] *= z;
        // d = u / u2
        const float inv = 1.0f / u[2];
        const float dot = (gd[0] * u[0] + gd[1] * u[1]) + gd[2] * u[2];
        float gu[3];
  #pragma unroll
        for (int b = 0; b < 3; ++b) gu[b] = gd[b] * inv;
        gu[2] -= dot * inv * inv;
        const float* Ki = cam + kOffKinv;
        gxy[0] = (Ki[0] * gu[0] + Ki[3] * gu[1]) + Ki[6] * gu[2];
        gxy[1] = (Ki[1] * gu[0] + Ki[4] * gu[1]) + Ki[7] * gu[2];
        if constexpr (GLUE) {
          dh[1] = gxy[0] * (1.0f / (float)a.W) * s1 * (1.0f - s1);
          dh[2] = gxy[1] * (1.0f / (float)a.H) * s2 * (1.0f - s2);
        }
      }
      // covariance -> scales, rotation
      {
        float sc[3], sraw[3];
  #pragma unroll
        for (int k = 0; k < 3; ++k) {
          sraw[k] = softplusf(h[O + k] - 4.0f);
          sc[k] = fminf(fmaxf(sraw[k], a.smin), a.smax);
        }
        float r[4], q[4];
  #pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = h[O + 3 + k];
        const float L = sqrtf(((r[0] * r[0] + r[1] * r[1]) + r[2] * r[2]) + r[3] * r[3]);
  #pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = r[k] / (L + a.eps);
        QuatR qr;
        quat_to_R(q, qr);
        float T[9], gC[9];
        mmt3(cam + kOffR, gCw, T);  // Rc^T gCw
        mm3(T, cam + kOffR, gC);    // (Rc^T gCw) Rc
        // C = R diag(s^2) R^T: dR = (gC + gC^T) R diag(s^2); dsig_k = (R^T gC R)_kk
        float gS[9], gR[9];
  #pragma unroll
        for (int k = 0; k < 9; ++k) gS[k] = gC[k] + gC[(k % 3) * 3 + k / 3];
        float RS2[9];
  #pragma unroll
        for (int i = 0; i < 3; ++i)
  #pragma unroll
          for (int k = 0; k < 3; ++k) RS2[i * 3 + k] = qr.R[i * 3 + k] * (sc[k] * sc[k]);
        mm3(gS, RS2, gR);
        float GR[9];
        mm3(gC, qr.R, GR);  // gC R
  #pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float dsig = (qr.R[k] * GR[k] + qr.R[3 + k] * GR[3 + k]) + qr.R[6 + k] * GR[6 + k];
          const float ds = 2.0f * sc[k] * dsig + gsc[k];  // + the scales output's own gradient
          const bool pass = sraw[k] >= a.smin && sraw[k] <= a.smax;  // torch.clamp gradient mask
          dh[O + k] = pass ? ds * softplus_grad(h[O + k] - 4.0f) : 0.0f;
        }
        // R(q) = I + s2 P(q), s2 = 2 / (|q|^2 + eps)
        const float i = q[0], j = q[1], kk = q[2], w = q[3], s2 = qr.s2;
        const float P[9] = {-(j * j + kk * kk), i * j - kk * w, i * kk + j * w,
                            i * j + kk * w,     -(i * i + kk * kk), j * kk - i * w,
                            i * kk - j * w,     j * kk + i * w,     -(i * i + j * j)};
        float gs2 = 0.f;
  #pragma unroll
        for (int k = 0; k < 9; ++k) gs2 += gR[k] * P[k];
        const float g = gR[0], g01 = gR[1], g02 = gR[2], g10 = gR[3], g11 = gR[4], g12 = gR[5], g20 = gR[6],
                    g21 = gR[7], g22 = gR[8];
        float gq[4];
        gq[0] = s2 * (g01 * j + g02 * kk + g10 * j - 2.f * g11 * i - g12 * w + g20 * kk + g21 * w - 2.f * g22 * i);
        gq[1] = s2 * (-2.f * g * j + g01 * i + g02 * w + g10 * i + g12 * kk - g20 * w + g21 * kk - 2.f * g22 * j);
        gq[2] = s2 * (-2.f * g * kk - g01 * w + g02 * i + g10 * w - 2.f * g11 * kk + g12 * j + g20 * i + g21 * j);
        gq[3] = s2 * (-g01 * kk + g02 * j + g10 * kk - g12 * i - g20 * j + g21 * i);
  #pragma unroll
        for (int m = 0; m < 4; ++m) gq[m] = gq[m] - gs2 * s2 * s2 * q[m] + grot[m];  // + rotations output grad
        // q = r / (|r| + eps)
        const float Le = L + a.eps;
        const float dqr = ((gq[0] * r[0] + gq[1] * r[1]) + gq[2] * r[2]) + gq[3] * r[3];
        const float c2 = L > 0.f ? dqr / (L * Le * Le) : 0.f;
  #pragma unroll
        for (int m = 0; m < 4; ++m) dh[O + 3 + m] = gq[m] / Le - c2 * r[m];
      }
      // harmonics -> raw SH: D^T per degree block, then the mask
  #pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* g2 = gh + c * NSH;
        float gs[NSH];
        gs[0] = g2[0];
  #pragma unroll
        for (int l = 1; l * l < NSH; ++l) {
          const int n = 2 * l + 1, b0 = l * l;
          const float* D = dblock<NSH>(cam, l);
  #pragma unroll
          for (int k = 0; k < n; ++k) {
            float acc = 0.f;
  #pragma unroll
            for (int i2 = 0; i2 < n; ++i2) acc += D[i2 * n + k] * g2[b0 + i2];
            gs[b0 + k] = acc;
          }
        }
  #pragma unroll
        for (int k = 0; k < NSH; ++k) dh[O + 7 + c * NSH + k] = gs[k] * a.sh_mask[k];
      }
}

}  // namespace dga
