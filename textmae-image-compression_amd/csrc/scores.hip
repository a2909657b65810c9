// Patch importance scores — the producer of MCM.forward's `total_scores` (reference
// generate_scores_file.py:19-31 over utils/map.py:6-60 and utils/distribution.py:5-16):
//   seg     = quadtree split / merge of the grayscale image, in place (Division_Merge_Segmented)
//   s_map   = resize(seg[1:-1, 1:-1], size x size)            INTER_LINEAR (cv2.resize)
//   t_map   = resize(|Laplacian_3x3(seg)| saturated, size^2)   (cv2.Laplacian ksize 3 + convertScaleAbs; the
//             reference takes the Laplacian of the image AFTER the merges, map.py:46-59 / generate_scores_file.py:22-23)
//   score   = int-mean(t_map 16x16 patch) * int-mean(s_map patch), min-max normalised (float64 -> float32)
// cv2 semantics as restated in oracle/scores_oracle.py (parity unpinned: OpenCV is not in the image); the
// kernels are bit-exact with that restatement.
//
// The quadtree runs level-synchronously with no host round trip: level l launches n * 4^l workgroups, one
// per potential block (the block geometry is the path of quadrant digits); a block whose parent did not
// split exits at once.  Every judgement reads the ORIGINAL pixels of its block: merges only touch leaf
// blocks, which never overlap a block judged later (children cover disjoint parts of their parent), so
// the in-place order of the reference's depth-first recursion (map.py:35-42) gives the same image.
#include <climits>

#include "common.h"

#define SC_THREADS 256

// geometry of block q at `level`: sizes halve (floor) per level, offsets add the quadrant digits
__device__ __forceinline__ void block_geom(int q, int level, int H, int W, int& h0, int& w0, int& h, int& w) {
  h0 = 0;
  w0 = 0;
  h = H;
  w = W;
  for (int l = level - 1; l >= 0; --l) {
    const int d = (q >> (2 * l)) & 3;  // quadrant chosen at depth (level - l): 0 TL, 1 TR, 2 BL, 3 BR
    const int h2 = h / 2, w2 = w / 2;
    if (d & 1) w0 += w2;
    if (d & 2) h0 += h2;
    h = h2;
    w = w2;
  }
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = SC_THREADS / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const T r = red[0];
  __syncthreads();
  return r;
}

// Division_Judge (map.py:6-23) + Recursion's split / Merge decision (map.py:35-42) for every live block
__global__ void __launch_bounds__(SC_THREADS)
quadtree_level_kernel(unsigned char* __restrict__ img, int H, int W, int level, const unsigned char* __restrict__ parent,
                      unsigned char* __restrict__ split) {
  __shared__ long long red[SC_THREADS];
  const long long nq = 1ll << (2 * level);
  const int b = (int)(blockIdx.x / nq);
  const int q = (int)(blockIdx.x - (long long)b * nq);
  unsigned char* im = img + (size_t)b * H * W;
  if (level > 0 && !parent[(size_t)b * (nq >> 2) + (q >> 2)]) {
    if (threadIdx.x == 0) split[blockIdx.x] = 0;
    return;
  }
  int h0, w0, h, w;
  block_geom(q, level, H, W, h0, w0, h, w);
  const long long n = (long long)h * w;
  long long s = 0, sxx = 0;
  for (int r = 0; r < h; ++r)
    for (int c = threadIdx.x; c < w; c += SC_THREADS) {
      const long long v = im[(size_t)(h0 + r) * W + w0 + c];
      s += v;
      sxx += v * v;
    }
  s = block_sum(s, red);
  sxx = block_sum(sxx, red);
  bool judged = false;
  if (n >= 2) {
    // (v - mean) < 2 std(ddof=1)  <=>  d < 0  or  d^2 (n - 1) < 4 n Q,  d = n v - S,  Q = n Sxx - S^2
    const __int128 rhs = (__int128)4 * n * (__int128)(n * sxx - s * s);
    long long ok = 0;
    for (int r = 0; r < h; ++r)
      for (int c = threadIdx.x; c < w; c += SC_THREADS) {
        const long long d = n * (long long)im[(size_t)(h0 + r) * W + w0 + c] - s;
        ok += (d < 0 || (__int128)d * d * (n - 1) < rhs) ? 1 : 0;
      }
    ok = block_sum(ok, red);
    judged = 20 * ok >= 19 * n;  // operated / total >= 0.95
  }
  const bool do_split = !judged && min(h, w) > 5;
  if (threadIdx.x == 0) split[blockIdx.x] = do_split ? 1 : 0;
  if (do_split) return;
  __syncthreads();  // every read of the block above happens before its merge below
  for (int r = 0; r < h; ++r)
    for (int c = threadIdx.x; c < w; c += SC_THREADS) {
      unsigned char* p = im + (size_t)(h0 + r) * W + w0 + c;
      const unsigned char v = *p;
      *p = (v > 60 && v < 150) ? 0 : 255;  // Merge (map.py:27-31)
    }
}

// |Laplacian ksize 3| saturated to uint8: aperture [[2,0,2],[0,-8,0],[2,0,2]], BORDER_REFLECT_101
__global__ void __launch_bounds__(SC_THREADS)
laplacian_abs_kernel(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst, int n, int H, int W) {
  const long long i = (long long)blockIdx.x * SC_THREADS + threadIdx.x;
  if (i >= (long long)n * H * W) return;
  const int b = (int)(i / ((long long)H * W));
  const int rem = (int)(i - (long long)b * H * W);
  const int y = rem / W, x = rem - y * W;
  const unsigned char* s = src + (size_t)b * H * W;
  auto rf = [](int v, int n_) { return v < 0 ? -v : (v >= n_ ? 2 * n_ - 2 - v : v); };
  const int ym = rf(y - 1, H), yp = rf(y + 1, H), xm = rf(x - 1, W), xp = rf(x + 1, W);
  const int lap = 2 * ((int)s[ym * W + xm] + s[ym * W + xp] + s[yp * W + xm] + s[yp * W + xp]) - 8 * (int)s[y * W + x];
  dst[i] = (unsigned char)min(lap < 0 ? -lap : lap, 255);
}

// cv2.resize INTER_LINEAR coefficient of destination index d (see oracle/scores_oracle.py): source index,
// 11-bit weights; `clamp` moves border taps onto the edge (columns), rows keep weights and clip the index
__device__ __forceinline__ void lin_coef(int d, int ssize, int dsize, bool clamp, int& s, int& a0, int& a1) {
#pragma clang fp contract(off)  // OpenCV's x86 build rounds the product and the difference separately
  const double scale = 1.0 / ((double)dsize / (double)ssize);
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  s = (int)floorf(f);
  f = f - (float)s;
  if (clamp && s < 0) { f = 0.0f; s = 0; }
  if (clamp && s >= ssize - 1) { f = 0.0f; s = ssize - 1; }
  a0 = (int)rintf((1.0f - f) * 2048.0f);
  a1 = (int)rintf(f * 2048.0f);
}

// dst[n][DH][DW] = resize(src[n][y0 : y0 + SH][x0 : x0 + SW] of a [H][W] plane); the vertical pass is the
// x86 vector kernel's arithmetic (VResizeLinearVec_32s8u)
__global__ void __launch_bounds__(SC_THREADS)
resize_linear_u8_kernel(const unsigned char* __restrict__ src, int H, int W, int y0, int x0, int SH, int SW,
                        unsigned char* __restrict__ dst, int n, int DH, int DW) {
  const long long i = (long long)blockIdx.x * SC_THREADS + threadIdx.x;
  if (i >= (long long)n * DH * DW) return;
  const int b = (int)(i / ((long long)DH * DW));
  const int rem = (int)(i - (long long)b * DH * DW);
  const int dy = rem / DW, dx = rem - dy * DW;
  int sx, a0, a1, sy, b0, b1;
  lin_coef(dx, SW, DW, true, sx, a0, a1);
  lin_coef(dy, SH, DH, false, sy, b0, b1);
  const int sx1 = min(sx + 1, SW - 1);
  const int r0 = min(max(sy, 0), SH - 1), r1 = min(max(sy + 1, 0), SH - 1);
  const unsigned char* p = src + (size_t)b * H * W + (size_t)y0 * W + x0;
  const int S0 = (int)p[(size_t)r0 * W + sx] * a0 + (int)p[(size_t)r0 * W + sx1] * a1;
  const int S1 = (int)p[(size_t)r1 * W + sx] * a0 + (int)p[(size_t)r1 * W + sx1] * a1;
  const int v = (((S0 >> 4) * b0) >> 16) + (((S1 >> 4) * b1) >> 16);
  dst[i] = (unsigned char)min(max((v + 2) >> 2, 0), 255);
}

// cal_patch_score of both maps (int(mean) of each 16x16 patch), product, min-max normalisation; one
// workgroup per image, thread p owns patch p
__global__ void __launch_bounds__(SC_THREADS)
patch_scores_kernel(const unsigned char* __restrict__ tmap, const unsigned char* __restrict__ smap, int S, int P,
                    float* __restrict__ scores) {
  __shared__ long long mn[SC_THREADS], mx[SC_THREADS];
  const int b = blockIdx.x;
  const int np = S / P, L = np * np;
  long long tot = 0;
  const bool act = threadIdx.x < L;
  if (act) {
    const int py = threadIdx.x / np, px = threadIdx.x - py * np;
    long long st = 0, ss = 0;
    for (int r = 0; r < P; ++r)
      for (int c = 0; c < P; ++c) {
        const size_t o = (size_t)b * S * S + (size_t)(py * P + r) * S + px * P + c;
        st += tmap[o];
        ss += smap[o];
      }
    tot = (st / (P * P)) * (ss / (P * P));
  }
  mn[threadIdx.x] = act ? tot : LLONG_MAX;
  mx[threadIdx.x] = act ? tot : LLONG_MIN;
  __syncthreads();
  for (int s = SC_THREADS / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      mn[threadIdx.x] = min(mn[threadIdx.x], mn[threadIdx.x + s]);
      mx[threadIdx.x] = max(mx[threadIdx.x], mx[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (act) scores[(size_t)b * L + threadIdx.x] = (float)((double)(tot - mn[0]) / (double)(mx[0] - mn[0]));
}

static int score_levels(int H, int W) {
  int l = 1, h = H, w = W;
  while (min(h, w) > 5) {  // a block splits only while min(h, w) > 5
    h /= 2;
    w /= 2;
    ++l;
  }
  return l;
}

static long long flags_bytes(int n, int levels) {
  long long t = 0;
  for (int l = 0; l < levels; ++l) t += (long long)n << (2 * l);
  return t;
}

extern "C" long long tmae_image_scores_workspace(int n, int H, int W, int size) {
  const long long planes = (long long)n * H * W;
  return 2 * planes + 2ll * n * size * size + flags_bytes(n, score_levels(H, W)) + 256;
}

extern "C" int tmae_image_scores(const unsigned char* gray, int n, int H, int W, int size, int patch,
                                 unsigned char* work, long long work_bytes, float* scores, void* stream) {
  TMAE_REQUIRE(gray && work && scores && n > 0 && H >= 3 && W >= 3 && size > 0 && patch > 0 && size % patch == 0,
               "tmae_image_scores: bad arguments");
  TMAE_REQUIRE((size / patch) * (size / patch) <= SC_THREADS, "tmae_image_scores: more than %d patches", SC_THREADS);
  TMAE_REQUIRE(work_bytes >= tmae_image_scores_workspace(n, H, W, size), "tmae_image_scores: workspace too small");
  const int levels = score_levels(H, W);
  TMAE_REQUIRE(levels <= 15, "tmae_image_scores: image too large");
  hipStream_t st = (hipStream_t)stream;
  const size_t planes = (size_t)n * H * W;
  unsigned char* seg = work;
  unsigned char* lap = seg + planes;
  unsigned char* smap = lap + planes;
  unsigned char* tmap = smap + (size_t)n * size * size;
  unsigned char* flags = tmap + (size_t)n * size * size;
  if (hipMemcpyAsync(seg, gray, planes, hipMemcpyDeviceToDevice, st) != hipSuccess) {
    tmae_set_error(TMAE_EHIP, "tmae_image_scores: copy failed");
    return TMAE_EHIP;
  }
  const unsigned char* parent = nullptr;
  unsigned char* cur = flags;
  for (int l = 0; l < levels; ++l) {
    const long long nb = (long long)n << (2 * l);
    hipLaunchKernelGGL(quadtree_level_kernel, dim3((unsigned)nb), dim3(SC_THREADS), 0, st, seg, H, W, l, parent, cur);
    parent = cur;
    cur += nb;
  }
  const unsigned g1 = (unsigned)((planes + SC_THREADS - 1) / SC_THREADS);
  hipLaunchKernelGGL(laplacian_abs_kernel, dim3(g1), dim3(SC_THREADS), 0, st, (const unsigned char*)seg, lap, n, H, W);
  const unsigned g2 = (unsigned)(((size_t)n * size * size + SC_THREADS - 1) / SC_THREADS);
  hipLaunchKernelGGL(resize_linear_u8_kernel, dim3(g2), dim3(SC_THREADS), 0, st, (const unsigned char*)seg, H, W, 1, 1,
                     H - 2, W - 2, smap, n, size, size);
  hipLaunchKernelGGL(resize_linear_u8_kernel, dim3(g2), dim3(SC_THREADS), 0, st, (const unsigned char*)lap, H, W, 0, 0,
                     H, W, tmap, n, size, size);
  hipLaunchKernelGGL(patch_scores_kernel, dim3(n), dim3(SC_THREADS), 0, st, (const unsigned char*)tmap,
                     (const unsigned char*)smap, size, patch, scores);
  TMAE_LAUNCH_CHECK("tmae_image_scores");
}
