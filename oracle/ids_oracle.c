/*
 * ORACLE — test infrastructure only.  CPU restatement of MCM.get_ids_shuffle
 * (reference models/Compression/MCM.py:364-423) + the ids_restore argsort of MCM.random_masking
 * (MCM.py:579-580).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this; the product path (libtmae.so) never does.
 *
 * It follows the reference statement by statement on plain arrays (a deliberately different
 * formulation from the GPU kernel, which sorts once and places indices by prefix scans):
 *   unique() -> quantile() -> bucketize() -> group means -> softmax -> round -> per-group sorted
 *   suffix with Python slice semantics -> Counter(first-appearance order) -> first-`freq` indices
 *   per value -> remaining indices ascending.
 * Float details pinned against torch 2.10 CPU (see tools/probe_torch_numerics.py):
 *   - quantile: ranks = q * (n-1) in f32, torch's lerp with a fused multiply-add;
 *   - mean: torch's cascade_sum order with an 8-wide vector (SumKernel.cpp), then / count;
 *   - softmax: exp rounded from double, sequential sum, multiply by the reciprocal.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t kPct[9] = {0x3dcccccdu, 0x3e4ccccdu, 0x3e99999au, 0x3ecccccdu, 0x3f000000u,
                                 0x3f19999au, 0x3f333333u, 0x3f4ccccdu, 0x3f666666u};

static float bits2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static int cmp_float(const void* a, const void* b) {
  float x = *(const float*)a, y = *(const float*)b;
  return (x > y) - (x < y);
}

/* torch CPU float sum order: cascade_sum -> vectorized_inner_sum / scalar_inner_sum ->
 * row_sum(ilp 4) -> multi_row_sum(4 levels, level_step 16) */
static void multi_row_sum(const float* x, int size, int w, float* out /* 4*w */) {
  const int NR = 4 * w;
  float acc[4][4 * 16];
  memset(acc, 0, sizeof(acc));
  int i = 0;
  while (i + 16 <= size) {
    for (int j = 0; j < 16; ++j, ++i)
      for (int e = 0; e < NR; ++e) acc[0][e] = acc[0][e] + x[i * NR + e];
    for (int j = 1; j < 4; ++j) {
      for (int e = 0; e < NR; ++e) {
        acc[j][e] = acc[j][e] + acc[j - 1][e];
        acc[j - 1][e] = 0.0f;
      }
      if ((i & (15 << (j * 4))) != 0) break;
    }
  }
  for (; i < size; ++i)
    for (int e = 0; e < NR; ++e) acc[0][e] = acc[0][e] + x[i * NR + e];
  for (int j = 1; j < 4; ++j)
    for (int e = 0; e < NR; ++e) acc[0][e] = acc[0][e] + acc[j][e];
  memcpy(out, acc[0], sizeof(float) * NR);
}

static void row_sum(const float* x, int rows, int w, float* res /* w */) {
  float part[4 * 16];
  const int size_ilp = rows / 4;
  multi_row_sum(x, size_ilp, w, part);
  for (int r = size_ilp * 4; r < rows; ++r)
    for (int l = 0; l < w; ++l) part[l] = part[l] + x[r * w + l];
  for (int k = 1; k < 4; ++k)
    for (int l = 0; l < w; ++l) part[l] = part[l] + part[k * w + l];
  memcpy(res, part, sizeof(float) * w);
}

float oracle_torch_sum_f32(const float* x, int n, int lanes) {
  float v[16];
  if (lanes > 1 && n >= lanes) {
    const int rows = n / lanes;
    row_sum(x, rows, lanes, v);
    float fin = 0.0f;
    for (int k = rows * lanes; k < n; ++k) fin = fin + x[k];
    for (int l = 0; l < lanes; ++l) fin = fin + v[l];
    return fin;
  }
  row_sum(x, n, 1, v);
  return v[0];
}

/* one image: scores[L] -> shuffle[L] */
static void ids_one(const float* s_in, int L, int K, int lanes, int64_t* shuffle, int64_t* restore) {
  float* s = (float*)malloc(sizeof(float) * L);
  float* u = (float*)malloc(sizeof(float) * L);
  int* cat = (int*)malloc(sizeof(int) * L);
  float* keep = (float*)malloc(sizeof(float) * 2 * L);
  float* vals = (float*)malloc(sizeof(float) * 2 * L);
  int* freq = (int*)malloc(sizeof(int) * 2 * L);
  float* tmp = (float*)malloc(sizeof(float) * L);
  char* used = (char*)calloc(L, 1);
  for (int i = 0; i < L; ++i) s[i] = (s_in[i] == 0.0f) ? 0.0f : s_in[i];

  /* total_score.unique() (sorted) */
  memcpy(u, s, sizeof(float) * L);
  qsort(u, L, sizeof(float), cmp_float);
  int n = 0;
  for (int i = 0; i < L; ++i)
    if (n == 0 || u[i] != u[n - 1]) u[n++] = u[i];

  /* torch.quantile(unique, percentiles) — linear interpolation */
  float thr[9];
  for (int t = 0; t < 9; ++t) {
    const float q = bits2f(kPct[t]);
    const float rank = q * (float)(n - 1);
    const int lo = (int)rank;
    const float w = rank - (float)lo;
    const int hi = (int)ceilf(rank);
    const float a = u[lo], c = u[hi], d = c - a;
    thr[t] = (fabsf(w) < 0.5f) ? fmaf(w, d, a) : fmaf(-d, 1.0f - w, c);
  }

  /* torch.bucketize(right=False) */
  for (int i = 0; i < L; ++i) {
    int c = 0;
    for (int t = 0; t < 9; ++t) c += thr[t] < s[i];
    cat[i] = c;
  }

  /* group means (index order within a group, as total_score[categories == g]) */
  float means[10];
  int cnt[10];
  for (int g = 0; g < 10; ++g) {
    int m = 0;
    for (int i = 0; i < L; ++i)
      if (cat[i] == g) tmp[m++] = s[i];
    cnt[g] = m;
    means[g] = oracle_torch_sum_f32(tmp, m, lanes) / (float)m;
  }

  /* keep_values = group 9 in index order */
  int nk = 0;
  for (int i = 0; i < L; ++i)
    if (cat[i] == 9) keep[nk++] = s[i];

  /* softmax(means[:9]) * (K - |group9|), round half-even, .int() */
  const int new_target = K - nk;
  int has_nan = 0;
  float mx = means[0];
  for (int g = 0; g < 9; ++g) {
    has_nan |= isnan(means[g]);
    if (means[g] > mx) mx = means[g];
  }
  float e[9], sum = 0.0f;
  for (int g = 0; g < 9; ++g) {
    e[g] = (float)exp((double)(means[g] - mx));
    sum = sum + e[g];
  }
  const float rs = 1.0f / sum;
  for (int g = 0; g < 9; ++g) {
    int32_t ntk = has_nan ? INT32_MIN : (int32_t)rintf((e[g] * rs) * (float)new_target);
    int m = 0;
    for (int i = 0; i < L; ++i)
      if (cat[i] == g) tmp[m++] = s[i];
    qsort(tmp, m, sizeof(float), cmp_float);
    /* start_index = len - num_to_keep as a 0-d int32 tensor (wraps), then group_score[start:] */
    const int64_t start = (int32_t)((uint32_t)m - (uint32_t)ntk);
    int64_t b = start >= 0 ? start : (int64_t)m + start;
    if (b < 0) b = 0;
    for (int64_t j = b; j < m; ++j) keep[nk++] = tmp[j];
  }

  /* Counter(keep_values): insertion order of distinct values, with counts */
  int nv = 0;
  for (int k = 0; k < nk; ++k) {
    int f = -1;
    for (int j = 0; j < nv; ++j)
      if (vals[j] == keep[k]) { f = j; break; }
    if (f < 0) { vals[nv] = keep[k]; freq[nv] = 1; ++nv; }
    else freq[f]++;
  }
  /* first `freq` indices where total_score == value */
  int out = 0;
  for (int j = 0; j < nv; ++j) {
    int taken = 0;
    for (int i = 0; i < L && taken < freq[j]; ++i)
      if (s[i] == vals[j]) { shuffle[out++] = i; used[i] = 1; ++taken; }
  }
  /* remaining indices ascending */
  for (int i = 0; i < L; ++i)
    if (!used[i]) shuffle[out++] = i;
  for (int j = 0; j < L; ++j) restore[shuffle[j]] = j;

  free(s); free(u); free(cat); free(keep); free(vals); free(freq); free(tmp); free(used);
}

/* returns 0, or 1 when K > L (the reference raises ValueError, MCM.py:374-376) */
int oracle_ids_shuffle(const float* scores, int N, int L, int K, int lanes, int64_t* shuffle, int64_t* restore) {
  if (K > L) return 1;
  for (int b = 0; b < N; ++b) ids_one(scores + (size_t)b * L, L, K, lanes, shuffle + (size_t)b * L, restore + (size_t)b * L);
  return 0;
}
