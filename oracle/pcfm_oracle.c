/*
 * pcfm_oracle.c -- CPU restatement of the reference's hot-path kernels.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (point-cloud-flow-
 * matching_amd/) loads or calls this file; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg do, and only as the checker / the timed CPU
 * baseline, never as a fallback.
 *
 * Each function restates the reference CUDA kernel named in its comment
 * (paths relative to the reference tree) as plain sequential C: one "thread"
 * after another in index order, so the float-atomic sums of the reference
 * (whose order is non-deterministic on the GPU) take the sequential order.
 *
 * Floating-point contract (shared with the HIP kernels, both built with
 * -ffp-contract=off and explicit fused multiply-adds):
 *   squared distance   d = fmaf(dz, dz, fmaf(dx, dx, dy*dy))   dx = q - p
 *   devox gather       a = w1*f1; a = fmaf(w0, f0, a); a = fmaf(wk, fk, a), k = 2..7
 *   sums of products   acc = fmaf(x, y, acc)   (nvcc contracts `acc += x*y`)
 * The reference CUDA cannot be built here (no nvcc / CUDA runtime; see
 * DESIGN.md "Oracle"), so these contracts are pinned against the reference's
 * own test fixtures where they exist (Chamfer: chamfer_python.distChamfer
 * outputs; EMD: test_emd_loss.py known answer) and are otherwise a restatement
 * of the .cu source: parity for the PVCNN kernels is pinned to the source text
 * plus hand-built known answers, not to executed reference outputs.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_API __attribute__((visibility("default")))

/* ---------------------------------------------------------------------- */
/* PVCNN voxelization: vox.cu:18-110                                       */
/* ---------------------------------------------------------------------- */

/* grid_stats_kernel (vox.cu:18-34) + avg_voxelize_kernel (vox.cu:48-72).
 * out/ind/cnt are fully written (the reference zero-fills them first). */
ORACLE_API void oracle_avg_voxelize_fwd(const float* feat, const int* coords, int b, int c,
                                        int n, int r, float* out, int* ind, int* cnt) {
  const int r2 = r * r, s = r2 * r;
  memset(out, 0, sizeof(float) * (size_t)b * c * s);
  memset(cnt, 0, sizeof(int) * (size_t)b * s);
  for (int bb = 0; bb < b; ++bb) {
    const int* cb = coords + (size_t)bb * 3 * n;
    int* ib = ind + (size_t)bb * n;
    int* kb = cnt + (size_t)bb * s;
    for (int i = 0; i < n; ++i) {
      ib[i] = cb[i] * r2 + cb[i + n] * r + cb[i + 2 * n];
      if (ib[i] >= 0 && ib[i] < s) kb[ib[i]] += 1;
    }
    const float* fb = feat + (size_t)bb * c * n;
    float* ob = out + (size_t)bb * c * s;
    for (int i = 0; i < n; ++i) {
      const int pos = ib[i];
      if (pos < 0 || pos >= s) continue;
      const int cur = kb[pos];
      if (cur > 0) {
        const float div = (float)(1.0 / (double)(float)cur);
        for (int j = 0; j < c; ++j) ob[(size_t)j * s + pos] += fb[(size_t)j * n + i] * div;
      }
    }
  }
}

/* avg_voxelize_grad_kernel (vox.cu:86-110): each (j, i) written once. */
ORACLE_API void oracle_avg_voxelize_bwd(const float* grad_y, const int* ind, const int* cnt,
                                        int b, int c, int n, int s, float* grad_x) {
  memset(grad_x, 0, sizeof(float) * (size_t)b * c * n);
  for (int bb = 0; bb < b; ++bb) {
    const int* ib = ind + (size_t)bb * n;
    const int* kb = cnt + (size_t)bb * s;
    const float* gy = grad_y + (size_t)bb * c * s;
    float* gx = grad_x + (size_t)bb * c * n;
    for (int i = 0; i < n; ++i) {
      const int pos = ib[i];
      if (pos < 0 || pos >= s) continue;
      const int cur = kb[pos];
      if (cur > 0) {
        const float div = (float)(1.0 / (double)(float)cur);
        for (int j = 0; j < c; ++j) gx[(size_t)j * n + i] += gy[(size_t)j * s + pos] * div;
      }
    }
  }
}

/* ---------------------------------------------------------------------- */
/* PVCNN trilinear devoxelization: trilinear_devox.cu:21-162               */
/* ---------------------------------------------------------------------- */

static void devox_corners(float x, float y, float z, int r, int idx[8], float w[8]) {
  const int r2 = r * r;
  const float xl = floorf(x), yl = floorf(y), zl = floorf(z);
  const float x1 = x - xl, y1 = y - yl, z1 = z - zl;
  const float x0 = 1.0f - x1, y0 = 1.0f - y1, z0 = 1.0f - z1;
  w[0] = x0 * y0 * z0;
  w[1] = x0 * y0 * z1;
  w[2] = x0 * y1 * z0;
  w[3] = x0 * y1 * z1;
  w[4] = x1 * y0 * z0;
  w[5] = x1 * y0 * z1;
  w[6] = x1 * y1 * z0;
  w[7] = x1 * y1 * z1;
  /* x_hi/y_hi sentinels: -1 & r2 == r2 when the fraction is > 0 (:64-75) */
  const int xh = (x1 > 0) ? -1 : 0, yh = (y1 > 0) ? -1 : 0, zh = (z1 > 0) ? 1 : 0;
  idx[0] = (int)xl * r2 + (int)yl * r + (int)zl;
  idx[1] = idx[0] + zh;
  idx[2] = idx[0] + (yh & r);
  idx[3] = idx[2] + zh;
  idx[4] = idx[0] + (xh & r2);
  idx[5] = idx[4] + zh;
  idx[6] = idx[4] + (yh & r);
  idx[7] = idx[6] + zh;
}

/* trilinear_devoxelize_kernel (:21-105).  inds/wgts [b, 8, n] written when
 * training != 0. */
ORACLE_API void oracle_trilinear_devoxelize_fwd(const float* coords, const float* feat, int b,
                                                int c, int n, int r, int training, float* out,
                                                int* inds, float* wgts) {
  const int s = r * r * r;
  for (int bb = 0; bb < b; ++bb) {
    const float* cb = coords + (size_t)bb * 3 * n;
    const float* fb = feat + (size_t)bb * c * s;
    float* ob = out + (size_t)bb * c * n;
    for (int i = 0; i < n; ++i) {
      int id[8];
      float w[8];
      devox_corners(cb[i], cb[i + n], cb[i + 2 * n], r, id, w);
      if (training) {
        for (int k = 0; k < 8; ++k) {
          inds[((size_t)bb * 8 + k) * n + i] = id[k];
          wgts[((size_t)bb * 8 + k) * n + i] = w[k];
        }
      }
      /* out-of-range corners (coords outside [0, r-1]) contribute 0 */
      for (int k = 0; k < 8; ++k)
        if (id[k] < 0 || id[k] >= s) {
          id[k] = 0;
          w[k] = 0.0f;
        }
      for (int j = 0; j < c; ++j) {
        const float* f = fb + (size_t)j * s;
        float a = w[1] * f[id[1]];
        a = fmaf(w[0], f[id[0]], a);
        for (int k = 2; k < 8; ++k) a = fmaf(w[k], f[id[k]], a);
        ob[(size_t)j * n + i] = a;
      }
    }
  }
}

/* trilinear_devoxelize_grad_kernel (:119-162), sequential atomics. */
ORACLE_API void oracle_trilinear_devoxelize_bwd(const float* grad_y, const int* inds,
                                                const float* wgts, int b, int c, int n, int r,
                                                float* grad_x) {
  const int s = r * r * r;
  memset(grad_x, 0, sizeof(float) * (size_t)b * c * s);
  for (int bb = 0; bb < b; ++bb) {
    const float* gy = grad_y + (size_t)bb * c * n;
    float* gx = grad_x + (size_t)bb * c * s;
    for (int i = 0; i < n; ++i) {
      int id[8];
      float w[8];
      for (int k = 0; k < 8; ++k) {
        id[k] = inds[((size_t)bb * 8 + k) * n + i];
        w[k] = wgts[((size_t)bb * 8 + k) * n + i];
      }
      for (int j = 0; j < c; ++j) {
        const float g = gy[(size_t)j * n + i];
        for (int k = 0; k < 8; ++k)
          if (id[k] >= 0 && id[k] < s) gx[(size_t)j * s + id[k]] += w[k] * g;
      }
    }
  }
}

/* ---------------------------------------------------------------------- */
/* Ball query (ball_query.cu:19-50) and grouping (grouping.cu:18-77)       */
/* ---------------------------------------------------------------------- */

ORACLE_API void oracle_ball_query(const float* centers, const float* points, int b, int m,
                                  int n, float radius, int u, int* idx) {
  const float r2 = radius * radius;
  memset(idx, 0, sizeof(int) * (size_t)b * m * u);
  for (int bb = 0; bb < b; ++bb) {
    const float* cb = centers + (size_t)bb * 3 * m;
    const float* pb = points + (size_t)bb * 3 * n;
    int* ob = idx + (size_t)bb * m * u;
    for (int j = 0; j < m; ++j) {
      const float cx = cb[j], cy = cb[j + m], cz = cb[j + 2 * m];
      for (int k = 0, cnt = 0; k < n && cnt < u; ++k) {
        const float dx = cx - pb[k], dy = cy - pb[k + n], dz = cz - pb[k + 2 * n];
        const float d2 = fmaf(dz, dz, fmaf(dx, dx, dy * dy));
        if (d2 < r2) {
          if (cnt == 0)
            for (int v = 0; v < u; ++v) ob[(size_t)j * u + v] = k;
          ob[(size_t)j * u + cnt] = k;
          ++cnt;
        }
      }
    }
  }
}

ORACLE_API void oracle_grouping_fwd(const float* feat, const int* idx, int b, int c, int n, int m,
                                    int u, float* out) {
  for (int bb = 0; bb < b; ++bb)
    for (int l = 0; l < c; ++l)
      for (int j = 0; j < m; ++j)
        for (int k = 0; k < u; ++k) {
          const int v = idx[((size_t)bb * m + j) * u + k];
          out[(((size_t)bb * c + l) * m + j) * u + k] =
              (v >= 0 && v < n) ? feat[((size_t)bb * c + l) * n + v] : 0.0f;
        }
}

ORACLE_API void oracle_grouping_bwd(const float* grad_y, const int* idx, int b, int c, int n,
                                    int m, int u, float* grad_x) {
  memset(grad_x, 0, sizeof(float) * (size_t)b * c * n);
  for (int bb = 0; bb < b; ++bb)
    for (int l = 0; l < c; ++l)
      for (int j = 0; j < m; ++j)
        for (int k = 0; k < u; ++k) {
          const int v = idx[((size_t)bb * m + j) * u + k];
          if (v >= 0 && v < n)
            grad_x[((size_t)bb * c + l) * n + v] += grad_y[(((size_t)bb * c + l) * m + j) * u + k];
        }
}

/* ---------------------------------------------------------------------- */
/* Chamfer-3D: chamfer3D.cu:12-195                                          */
/* ---------------------------------------------------------------------- */

static void nn_dir(const float* q, int nq, const float* p, int np, int b, float* dist, int* idx) {
  for (int bb = 0; bb < b; ++bb)
    for (int j = 0; j < nq; ++j) {
      const float* a = q + ((size_t)bb * nq + j) * 3;
      float best = 0.0f;
      int bi = 0;
      for (int k = 0; k < np; ++k) {
        const float* c = p + ((size_t)bb * np + k) * 3;
        const float dx = c[0] - a[0], dy = c[1] - a[1], dz = c[2] - a[2];
        const float d = fmaf(dz, dz, fmaf(dx, dx, dy * dy));
        if (k == 0 || d < best) { /* first candidate always taken (:36, :121) */
          best = d;
          bi = k;
        }
      }
      dist[(size_t)bb * nq + j] = best; /* np == 0: stays the zero fill */
      idx[(size_t)bb * nq + j] = bi;
    }
}

ORACLE_API void oracle_chamfer_fwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                                   float* dist1, float* dist2, int* idx1, int* idx2) {
  nn_dir(xyz1, n, xyz2, m, b, dist1, idx1);
  nn_dir(xyz2, m, xyz1, n, b, dist2, idx2);
}

/* NmDistanceGradKernel: accumulates, like the reference (callers zero). */
ORACLE_API void oracle_chamfer_bwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                                   const float* gd1, const float* gd2, const int* idx1,
                                   const int* idx2, float* g1, float* g2) {
  for (int dir = 0; dir < 2; ++dir) {
    const float* qp = dir ? xyz2 : xyz1;
    const float* cp = dir ? xyz1 : xyz2;
    const float* gd = dir ? gd2 : gd1;
    const int* ix = dir ? idx2 : idx1;
    float* gq = dir ? g2 : g1;
    float* gc = dir ? g1 : g2;
    const int nq = dir ? m : n, nc = dir ? n : m;
    for (int bb = 0; bb < b; ++bb)
      for (int j = 0; j < nq; ++j) {
        const size_t o = (size_t)bb * nq + j;
        const int j2 = ix[o];
        if (j2 < 0 || j2 >= nc) continue;
        const float* a = qp + o * 3;
        const float* c = cp + ((size_t)bb * nc + j2) * 3;
        const float g = gd[o] * 2.0f;
        for (int x = 0; x < 3; ++x) {
          const float t = g * (a[x] - c[x]);
          gq[o * 3 + x] += t;
          gc[((size_t)bb * nc + j2) * 3 + x] -= t;
        }
      }
  }
}

/* ---------------------------------------------------------------------- */
/* Approximate EMD: emd_kernel.cu:24-353, one block's sequential view.      */
/* ---------------------------------------------------------------------- */

#define EMD_BODY(T, FMA)                                                                       \
  const int nn_ = n, mm_ = m;                                                                  \
  memset(match, 0, sizeof(T) * (size_t)b * m * n);                                             \
  if (n == 0 || m == 0) return;                                                                \
  T* remL = (T*)malloc(sizeof(T) * (size_t)(2 * n + 2 * m));                                   \
  T* remR = remL + n;                                                                          \
  T* ratL = remR + m;                                                                          \
  T* ratR = ratL + n;                                                                          \
  const T multiL = n >= m ? (T)1 : (T)(m / n);                                                 \
  const T multiR = n >= m ? (T)(n / m) : (T)1;                                                 \
  for (int bb = 0; bb < b; ++bb) {                                                             \
    const T* p1 = xyz1 + (size_t)bb * nn_ * 3;                                                 \
    const T* p2 = xyz2 + (size_t)bb * mm_ * 3;                                                 \
    T* mt = match + (size_t)bb * nn_ * mm_;                                                    \
    for (int k = 0; k < n; ++k) remL[k] = multiL;                                              \
    for (int l = 0; l < m; ++l) remR[l] = multiR;                                              \
    for (int j = 7; j >= -2; --j) {                                                            \
      T level = (T)(-powf(4.0f, (float)j));                                                    \
      if (j == -2) level = 0;                                                                  \
      for (int k = 0; k < n; ++k) {                                                            \
        T suml = (T)1e-9f;                                                                     \
        for (int l = 0; l < m; ++l) {                                                          \
          const T dx = p2[l * 3] - p1[k * 3], dy = p2[l * 3 + 1] - p1[k * 3 + 1],              \
                  dz = p2[l * 3 + 2] - p1[k * 3 + 2];                                          \
          const T d = level * FMA(dz, dz, FMA(dx, dx, dy * dy));                               \
          suml = FMA((T)expf((float)d), remR[l], suml);                                        \
        }                                                                                      \
        ratL[k] = remL[k] / suml;                                                              \
      }                                                                                        \
      for (int l = 0; l < m; ++l) {                                                            \
        T sumr = 0;                                                                            \
        for (int k = 0; k < n; ++k) {                                                          \
          const T dx = p2[l * 3] - p1[k * 3], dy = p2[l * 3 + 1] - p1[k * 3 + 1],              \
                  dz = p2[l * 3 + 2] - p1[k * 3 + 2];                                          \
          sumr = FMA((T)expf((float)(level * FMA(dz, dz, FMA(dx, dx, dy * dy)))), ratL[k],     \
                     sumr);                                                                    \
        }                                                                                      \
        sumr *= remR[l];                                                                       \
        const T cons = (T)fminf((float)(remR[l] / (sumr + (T)1e-9f)), 1.0f);                   \
        ratR[l] = cons * remR[l];                                                              \
        remR[l] = (T)fmaxf(0.0f, (float)(remR[l] - sumr));                                     \
      }                                                                                        \
      for (int k = 0; k < n; ++k) {                                                            \
        T suml = 0;                                                                            \
        const T rl = ratL[k];                                                                  \
        for (int l = 0; l < m; ++l) {                                                          \
          const T dx = p2[l * 3] - p1[k * 3], dy = p2[l * 3 + 1] - p1[k * 3 + 1],              \
                  dz = p2[l * 3 + 2] - p1[k * 3 + 2];                                          \
          const T e = (T)expf((float)(level * FMA(dz, dz, FMA(dx, dx, dy * dy))));              \
          const T w = (e * rl) * ratR[l];                                                      \
          mt[(size_t)l * n + k] += w;                                                          \
          suml = FMA(e * rl, ratR[l], suml);                                                   \
        }                                                                                      \
        remL[k] = (T)fmaxf(0.0f, (float)(remL[k] - suml));                                     \
      }                                                                                        \
    }                                                                                          \
  }                                                                                            \
  free(remL);

ORACLE_API void oracle_emd_approxmatch_f32(const float* xyz1, const float* xyz2, int b, int n,
                                           int m, float* match) {
  EMD_BODY(float, fmaf)
}
ORACLE_API void oracle_emd_approxmatch_f64(const double* xyz1, const double* xyz2, int b, int n,
                                           int m, double* match) {
  EMD_BODY(double, fma)
}

#define COST_BODY(T, FMA)                                                                      \
  for (int bb = 0; bb < b; ++bb) {                                                             \
    T tot = 0;                                                                                 \
    for (int k = 0; k < n; ++k) {                                                              \
      T sub = 0;                                                                               \
      const T* a = xyz1 + ((size_t)bb * n + k) * 3;                                            \
      for (int l = 0; l < m; ++l) {                                                            \
        const T* c = xyz2 + ((size_t)bb * m + l) * 3;                                          \
        const T dx = c[0] - a[0], dy = c[1] - a[1], dz = c[2] - a[2];                          \
        sub = FMA(FMA(dz, dz, FMA(dx, dx, dy * dy)), match[((size_t)bb * m + l) * n + k], sub); \
      }                                                                                        \
      tot += sub;                                                                              \
    }                                                                                          \
    cost[bb] = tot;                                                                            \
  }

ORACLE_API void oracle_emd_matchcost_f32(const float* xyz1, const float* xyz2, const float* match,
                                         int b, int n, int m, float* cost) {
  COST_BODY(float, fmaf)
}
ORACLE_API void oracle_emd_matchcost_f64(const double* xyz1, const double* xyz2,
                                         const double* match, int b, int n, int m, double* cost) {
  COST_BODY(double, fma)
}

/* matchcostgrad1 (:332-353) / matchcostgrad2 (:285-325) */
#define GRAD_BODY(T, FMA)                                                                      \
  for (int bb = 0; bb < b; ++bb) {                                                             \
    const T g = gcost[bb];                                                                     \
    for (int k = 0; k < n; ++k) {                                                              \
      const T* a = xyz1 + ((size_t)bb * n + k) * 3;                                            \
      T d3[3] = {0, 0, 0};                                                                     \
      for (int l = 0; l < m; ++l) {                                                            \
        const T* c = xyz2 + ((size_t)bb * m + l) * 3;                                          \
        const T d = match[((size_t)bb * m + l) * n + k] * (T)2;                                \
        for (int x = 0; x < 3; ++x) d3[x] = FMA(a[x] - c[x], d, d3[x]);                        \
      }                                                                                        \
      for (int x = 0; x < 3; ++x) grad1[((size_t)bb * n + k) * 3 + x] = d3[x] * g;             \
    }                                                                                          \
    for (int l = 0; l < m; ++l) {                                                              \
      const T* c = xyz2 + ((size_t)bb * m + l) * 3;                                            \
      T d3[3] = {0, 0, 0};                                                                     \
      for (int k = 0; k < n; ++k) {                                                            \
        const T* a = xyz1 + ((size_t)bb * n + k) * 3;                                          \
        const T d = match[((size_t)bb * m + l) * n + k] * (T)2;                                \
        for (int x = 0; x < 3; ++x) d3[x] = FMA(c[x] - a[x], d, d3[x]);                        \
      }                                                                                        \
      for (int x = 0; x < 3; ++x) grad2[((size_t)bb * m + l) * 3 + x] = d3[x] * g;             \
    }                                                                                          \
  }

ORACLE_API void oracle_emd_matchcost_bwd_f32(const float* gcost, const float* xyz1,
                                             const float* xyz2, const float* match, int b, int n,
                                             int m, float* grad1, float* grad2) {
  GRAD_BODY(float, fmaf)
}
ORACLE_API void oracle_emd_matchcost_bwd_f64(const double* gcost, const double* xyz1,
                                             const double* xyz2, const double* match, int b,
                                             int n, int m, double* grad1, double* grad2) {
  GRAD_BODY(double, fma)
}
