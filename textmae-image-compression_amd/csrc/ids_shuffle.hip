// Patch-index generation on the GPU: one workgroup per image.
//
// Replaces MCM.get_ids_shuffle (reference models/Compression/MCM.py:364-423) and the
// argsort / keep-slice of MCM.random_masking (MCM.py:579-583).  The reference runs this as a
// per-sample Python loop with ~15 device<->host syncs per image; here the whole batch is one
// launch, nothing leaves HBM, and the result is bit-exact with the reference's integer output.
//
// Semantics reproduced (reference line -> what the kernel does):
//   381-384  thresholds = torch.quantile(unique(s), [0.1..0.9] f32): ranks = q*(n-1) in f32,
//            lerp with torch's contracted-FMA scalar formula
//   387      categories = bucketize(s, thresholds, right=False) = #thresholds strictly below s
//   390-393  group means in float32 with torch's CPU cascade-sum order (vector width `lanes`);
//            empty group -> NaN
//   399-402  scaled = round_half_even(softmax(means[:9]) * (K - |group9|)).int(); NaN -> INT_MIN
//   405-408  per group, the sorted suffix `[len - n:]` with Python slice semantics (negative
//            start wraps, int32 overflow of len - INT_MIN wraps exactly like the 0-d int32 tensor)
//   410-416  Counter insertion order: group-9 values in first-index order, then groups 0..8 in
//            ascending value order; each value contributes its first `freq` indices
//   418-420  remaining indices ascending
//
// Algorithm (all in LDS): bitonic sort of (value, index) keys; runs of equal values; per-group
// ranges are contiguous in sorted order because bucketize is monotone; three block scans place
// every index.  softmax uses exp rounded from double + sequential sum + reciprocal multiply
// (identical to the oracle bit-for-bit; vs torch's Sleef exp this can only differ
// when softmax*target lands within a few ulp of .5 — 0 of 3.6M sampled groups).
#include "sort.h"

#define IDS_MAXL 1024
#define IDS_THREADS 256
#define IDS_GROUPS 10

// torch.arange(0.1, 0.91, 0.1, dtype=float32) bit patterns (MCM.py:381)
__constant__ unsigned kPercentileBits[9] = {0x3dcccccdu, 0x3e4ccccdu, 0x3e99999au, 0x3ecccccdu, 0x3f000000u,
                                            0x3f19999au, 0x3f333333u, 0x3f4ccccdu, 0x3f666666u};


// ---- torch CPU float32 sum order (aten SumKernel.cpp cascade_sum / multi_row_sum / row_sum).
// acc: 4 levels x 4 ilp rows x W lanes scratch (LDS).  Valid for n <= 65536 (level_power = 4).
__device__ float torch_cascade_sum(const float* x, int n, int W, float* acc) {
  const int ilp = 4;
  const bool vec = (W > 1) && (n >= W);
  const int w = vec ? W : 1;
  const int rows = vec ? (n / W) : n;  // "size" passed to row_sum (vectors or scalars)
  const int size_ilp = rows / ilp;
  const int NR = ilp * w;
  for (int i = 0; i < 4 * NR; ++i) acc[i] = 0.0f;
  auto addrow = [&](float* dst, int r) {  // dst[k*w + l] += element (r*ilp + k, lane l)
    for (int k = 0; k < ilp; ++k)
      for (int l = 0; l < w; ++l) dst[k * w + l] = dst[k * w + l] + x[(r * ilp + k) * w + l];
  };
  int i = 0;
  while (i + 16 <= size_ilp) {
    for (int j = 0; j < 16; ++j, ++i) addrow(acc, i);
    for (int j = 1; j < 4; ++j) {
      for (int e = 0; e < NR; ++e) {
        acc[j * NR + e] = acc[j * NR + e] + acc[(j - 1) * NR + e];
        acc[(j - 1) * NR + e] = 0.0f;
      }
      if ((i & (15 << (j * 4))) != 0) break;
    }
  }
  for (; i < size_ilp; ++i) addrow(acc, i);
  for (int j = 1; j < 4; ++j)
    for (int e = 0; e < NR; ++e) acc[e] = acc[e] + acc[j * NR + e];
  // row_sum tail + fold of the ilp partials
  for (int r = size_ilp * ilp; r < rows; ++r)
    for (int l = 0; l < w; ++l) acc[l] = acc[l] + x[r * w + l];
  for (int k = 1; k < ilp; ++k)
    for (int l = 0; l < w; ++l) acc[l] = acc[l] + acc[k * w + l];
  if (!vec) return acc[0];
  float fin = 0.0f;
  for (int k = rows * W; k < n; ++k) fin = fin + x[k];
  for (int l = 0; l < W; ++l) fin = fin + acc[l];
  return fin;
}

// exclusive scan of `n` ints in LDS (n <= IDS_MAXL), returns total.  All threads call.  Each thread sums its chunk,
// the chunk sums are scanned inside each wave by lane shuffles and across the waves through tmp (two barriers;
// a Hillis-Steele scan over the workgroup took 16).  Integer sums: the same result in any order.
__device__ int block_exclusive_scan(int* a, int n, int* tmp /*IDS_THREADS / 64*/) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  constexpr int NWV = IDS_THREADS / 64;
  const int per = (n + IDS_THREADS - 1) / IDS_THREADS;
  const int beg = min(n, t * per), end = min(n, beg + per);
  int s = 0;
  for (int i = beg; i < end; ++i) s += a[i];
  int x = s;  // inclusive scan of the chunk sums within the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) tmp[wave] = x;
  __syncthreads();
  int run = x - s, total = 0;
#pragma unroll
  for (int w = 0; w < NWV; ++w) {
    const int tw = tmp[w];
    run += w < wave ? tw : 0;
    total += tw;
  }
  for (int i = beg; i < end; ++i) {
    const int v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

__global__ void __launch_bounds__(IDS_THREADS)
ids_shuffle_kernel(const float* __restrict__ scores, int64_t* __restrict__ ids_shuffle,
                   int64_t* __restrict__ ids_restore, int L, int P, int K, int lanes) {
  __shared__ unsigned long long key[IDS_MAXL];
  __shared__ float sv[IDS_MAXL];        // original scores (by index)
  __shared__ int cat_idx[IDS_MAXL];     // category by index
  __shared__ int sel_idx[IDS_MAXL];     // selected flag by index
  __shared__ int rid[IDS_MAXL];         // run id by sorted position (inclusive scan of flags)
  __shared__ int aux[IDS_MAXL];         // scratch: flags / scans
  __shared__ int runstart[IDS_MAXL];    // sorted position of each run's first element
  __shared__ int runpos9[IDS_MAXL];     // output offset of each group-9 run
  __shared__ int pos9[IDS_MAXL];        // by index: size of the group-9 run starting there (then its offset)
  __shared__ float glist[IDS_MAXL];     // scores compacted by (group, index)
  __shared__ float gacc[IDS_GROUPS][4 * 4 * 16];
  __shared__ int scan_tmp[IDS_THREADS];
  __shared__ int gcnt[IDS_GROUPS], goff[IDS_GROUPS], gbeg[IDS_GROUPS];
  __shared__ int wcnt[IDS_THREADS / 64][IDS_GROUPS];  // per wave: indices of each group (the compaction's ranks)
  __shared__ float gmean[IDS_GROUPS];
  __shared__ float e9[9];
  __shared__ float thr[9];
  __shared__ int keep[9];
  __shared__ int nuniq, cnt9, nsel_other;

  const int b = blockIdx.x, t = threadIdx.x;
  const float* s = scores + (size_t)b * L;

  // 1. load; canonicalise -0.0 so equal floats get equal keys (torch treats -0.0 == 0.0)
  for (int i = t; i < P; i += IDS_THREADS) {
    if (i < L) {
      float v = s[i];
      if (v == 0.0f) v = 0.0f;
      sv[i] = v;
      key[i] = ((unsigned long long)f2key(v) << 32) | (unsigned)i;
    } else {
      key[i] = ~0ull;
    }
  }
  if (t < IDS_GROUPS) gcnt[t] = 0;
  __syncthreads();

  // 2. bitonic sort ascending by (value, index)
  if (P <= IDS_THREADS) reg_bitonic_sort<IDS_THREADS>(key, P);
  else lds_bitonic_sort<IDS_THREADS>(key, P);

  // 3. runs of equal values (float equality)
  for (int p = t; p < L; p += IDS_THREADS) {
    float v = key2f((unsigned)(key[p] >> 32));
    int flag = (p == 0) ? 1 : (v != key2f((unsigned)(key[p - 1] >> 32)));
    aux[p] = flag;
    rid[p] = flag;
  }
  __syncthreads();
  int nu = block_exclusive_scan(rid, L, scan_tmp);  // rid = exclusive count of run starts
  for (int p = t; p < L; p += IDS_THREADS) {
    if (aux[p]) runstart[rid[p]] = p;
    else rid[p] -= 1;  // exclusive scan -> id of the run this element belongs to
  }
  if (t == 0) nuniq = nu;
  __syncthreads();

  // 4. thresholds = quantile(unique, q) with torch's float32 linear interpolation (MCM.py:383)
  if (t < 9) {
    const float q = __uint_as_float(kPercentileBits[t]);
    const int n = nuniq;
    float rank = q * (float)(n - 1);
    int lo = (int)rank;                 // ranks.toType(kLong)
    float w = rank - (float)lo;
    int hi = (int)ceilf(rank);
    float a = key2f((unsigned)(key[runstart[lo]] >> 32));
    float c = key2f((unsigned)(key[runstart[hi]] >> 32));
    float d = c - a;
    thr[t] = (fabsf(w) < 0.5f) ? __fmaf_rn(w, d, a) : __fmaf_rn(-d, 1.0f - w, c);
  }
  __syncthreads();

  // 5. categories (bucketize right=False) and group sizes
  for (int i = t; i < L; i += IDS_THREADS) {
    float v = sv[i];
    int c = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) c += (thr[k] < v) ? 1 : 0;
    cat_idx[i] = c;
    atomicAdd(&gcnt[c], 1);
  }
  __syncthreads();
  if (t == 0) {
    int o = 0;
    for (int g = 0; g < IDS_GROUPS; ++g) { goff[g] = o; o += gcnt[g]; }
  }
  __syncthreads();
  // compact scores by (group, index): rank within group = #earlier indices of the same group
  if (L <= IDS_THREADS) {
    // one index per thread: per-group ballots give the rank inside the wave, per-wave counts the waves before
    const int lane = t & 63, wave = t >> 6;
    const int c = t < L ? cat_idx[t] : -1;
    unsigned long long mine = 0;
#pragma unroll
    for (int g = 0; g < IDS_GROUPS; ++g) {
      const unsigned long long bm = __ballot(c == g);
      if (lane == 0) wcnt[wave][g] = __popcll(bm);
      if (c == g) mine = bm;
    }
    __syncthreads();
    if (c >= 0) {
      int r = __popcll(mine & ((1ull << lane) - 1ull));
      for (int w = 0; w < wave; ++w) r += wcnt[w][c];
      glist[goff[c] + r] = sv[t];
    }
  } else {
    for (int i = t; i < L; i += IDS_THREADS) {
      int c = cat_idx[i], r = 0;
      for (int j = 0; j < i; ++j) r += (cat_idx[j] == c);
      glist[goff[c] + r] = sv[i];
    }
  }
  __syncthreads();

  // 6. group means in torch's summation order (MCM.py:390-393)
  if (t < IDS_GROUPS) {
    float sum = torch_cascade_sum(glist + goff[t], gcnt[t], lanes, gacc[t]);
    gmean[t] = sum / (float)gcnt[t];  // 0/0 -> NaN for an empty group
  }
  __syncthreads();

  // 7. softmax over groups 0..8, scaled targets (MCM.py:399-402), slice lengths (MCM.py:405-408); the nine
  //    exponentials (rounded from double) in parallel, everything order-dependent on one thread
  if (t < 9) {
    float m = gmean[0];
    for (int g = 0; g < 9; ++g) m = fmaxf(m, gmean[g]);
    e9[t] = (float)exp((double)(gmean[t] - m));
  }
  __syncthreads();
  if (t == 0) {
    int c9 = gcnt[9];
    cnt9 = c9;
    int new_target = K - c9;
    bool has_nan = false;
    for (int g = 0; g < 9; ++g) has_nan |= isnan(gmean[g]);
    float e[9];
    float sum = 0.0f;
    for (int g = 0; g < 9; ++g) { e[g] = e9[g]; sum = sum + e[g]; }
    float rs = 1.0f / sum;
    int beg = 0;
    for (int g = 0; g < 9; ++g) {
      int ntk;
      if (has_nan) {
        ntk = (int)0x80000000;  // round(NaN).int() on x86
      } else {
        float sc = (e[g] * rs) * (float)new_target;
        ntk = (int)rintf(sc);
      }
      int len = gcnt[g];
      const long long start = (int)((unsigned)len - (unsigned)ntk);  // 0-d int32 tensor arithmetic wraps
      // Python slice group[start:]: negative start counts from the end, clamped at 0
      const int kept = (int)((start >= 0) ? (start >= len ? 0 : len - start) : (-start > len ? len : -start));
      keep[g] = kept;
      gbeg[g] = beg;
      beg += len;
    }
    gbeg[9] = beg;
  }
  __syncthreads();

  // 8. selection per sorted position.  Group g occupies sorted positions [gbeg[g], gbeg[g]+gcnt[g]).
  //    A run inside group g<9 contributes c = |run ∩ suffix| indices: its first c (lowest) indices.
  for (int p = t; p < L; p += IDS_THREADS) {
    int idx = (int)(key[p] & 0xffffffffu);
    int g = cat_idx[idx];
    int sel;
    if (g == 9) {
      sel = 1;
    } else {
      int ge = gbeg[g] + gcnt[g];
      int sb = ge - keep[g];
      int r = rid[p];
      int rs0 = runstart[r];
      int re = (r + 1 < nuniq) ? runstart[r + 1] : L;
      int c = max(0, min(re, ge) - max(rs0, sb));
      sel = (p - rs0) < c;
    }
    sel_idx[idx] = sel;
    aux[p] = (g != 9 && sel) ? 1 : 0;  // selected, non-group-9, by sorted position
  }
  __syncthreads();
  // group-9 runs ordered by their minimum index (= the index at the run's start): each run's size placed at that
  // index, an exclusive scan in index order gives every run its output offset (one O(L) scan; the pairwise count
  // over all runs was 2/3 of the kernel's time)
  for (int i = t; i < L; i += IDS_THREADS) pos9[i] = 0;
  __syncthreads();
  for (int r = t; r < nuniq; r += IDS_THREADS) {
    const int p0 = runstart[r];
    const int idx0 = (int)(key[p0] & 0xffffffffu);
    if (cat_idx[idx0] == 9) pos9[idx0] = ((r + 1 < nuniq) ? runstart[r + 1] : L) - p0;
  }
  __syncthreads();
  block_exclusive_scan(pos9, L, scan_tmp);
  for (int r = t; r < nuniq; r += IDS_THREADS) {
    const int idx0 = (int)(key[runstart[r]] & 0xffffffffu);
    if (cat_idx[idx0] == 9) runpos9[r] = pos9[idx0];
  }
  int nsel = block_exclusive_scan(aux, L, scan_tmp);  // aux = output rank among selected non-9
  if (t == 0) nsel_other = nsel;
  __syncthreads();

  int64_t* shuf = ids_shuffle + (size_t)b * L;
  int64_t* rest = ids_restore + (size_t)b * L;
  for (int p = t; p < L; p += IDS_THREADS) {
    int idx = (int)(key[p] & 0xffffffffu);
    int g = cat_idx[idx];
    int out = -1;
    if (g == 9) {
      int r = rid[p];
      out = runpos9[r] + (p - runstart[r]);
    } else if (sel_idx[idx]) {
      out = cnt9 + aux[p];
    }
    if (out >= 0) { shuf[out] = idx; rest[idx] = out; }
  }
  __syncthreads();
  // 9. unselected indices ascending after the selected ones (MCM.py:418-420)
  for (int i = t; i < L; i += IDS_THREADS) aux[i] = sel_idx[i] ? 0 : 1;
  __syncthreads();
  block_exclusive_scan(aux, L, scan_tmp);
  const int base = cnt9 + nsel_other;
  for (int i = t; i < L; i += IDS_THREADS) {
    if (!sel_idx[i]) { int out = base + aux[i]; shuf[out] = i; rest[i] = out; }
  }
}

extern "C" int tmae_ids_shuffle(const float* scores, int64_t* ids_shuffle, int64_t* ids_restore, int n, int L,
                                int K, int sum_lanes, void* stream) {
  TMAE_REQUIRE(n >= 0 && L >= 1 && L <= IDS_MAXL, "tmae_ids_shuffle: L=%d must be in [1, %d]", L, IDS_MAXL);
  TMAE_REQUIRE(K >= 0 && K <= L, "Number of patches should not be greater than the length of scores (K=%d, L=%d)", K, L);
  TMAE_REQUIRE(sum_lanes == 1 || sum_lanes == 8 || sum_lanes == 16, "tmae_ids_shuffle: sum_lanes must be 1, 8 or 16");
  if (n == 0) return TMAE_OK;
  int P = 1;
  while (P < L) P <<= 1;
  hipLaunchKernelGGL(ids_shuffle_kernel, dim3(n), dim3(IDS_THREADS), 0, (hipStream_t)stream, scores, ids_shuffle,
                     ids_restore, L, P, K, sum_lanes);
  TMAE_LAUNCH_CHECK("tmae_ids_shuffle");
}
