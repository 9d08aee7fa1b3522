// Retrieval: fused similarity GEMM + row top-k, top-k merge, recall counting.
//
// Reference path: scores = torch.matmul(txt.float(), img.float().t()) on the
// CPU (main.py:473, 100 MB / 500 MB fp32 matrices), then one torch.topk per
// row in a Python loop (main.py:331-378). Here the bf16 x bf16 -> fp32 MFMA
// GEMM of gemm_core.h feeds a top-k epilogue: each 128 x 128 score tile is
// spilled to LDS once and scanned by 2 threads per row that keep a sorted
// (score desc, column asc) list in registers. The score matrix never reaches
// HBM; per (row, column-split, half) candidate lists go to the workspace and a
// one-wave-per-row merge produces the final top-k.
#include "gemm_core.h"

namespace {
using namespace gemmcore;

constexpr int KMAX = 16;
using SimCfg = Cfg<128, 128, 2, 2>;
constexpr int TILE_LD = 128 + 4;  // fp32 score tile row stride in LDS
constexpr int SIM_LDS = (SimCfg::LDS > 128 * TILE_LD * 4) ? SimCfg::LDS : 128 * TILE_LD * 4;

// Insert (v, idx) into a sorted-desc list; strictly-greater keeps the earlier
// column first on ties (columns are scanned in increasing order).
__device__ __forceinline__ void topk_insert(float (&ts)[KMAX], int (&ti)[KMAX], float v, int idx) {
    if (!(v > ts[KMAX - 1])) return;
    ts[KMAX - 1] = v;
    ti[KMAX - 1] = idx;
#pragma unroll
    for (int j = KMAX - 1; j > 0; --j) {
        if (ts[j] > ts[j - 1]) {
            const float tv = ts[j];
            ts[j] = ts[j - 1];
            ts[j - 1] = tv;
            const int tx = ti[j];
            ti[j] = ti[j - 1];
            ti[j - 1] = tx;
        }
    }
}

struct SimArgs {
    const bf16* Q;
    const bf16* Dm;
    int ldq, ldd, nq, nd, D, k, col_offset;
    int tiles_per_split, nsplit;
    float* cand_s;  // [nq][nsplit*2][k]
    int* cand_i;
};

__global__ __launch_bounds__(SimCfg::NT) void sim_topk_kernel(SimArgs p) {
    __shared__ __attribute__((aligned(16))) char lds[SIM_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / SimCfg::WN, wn = wave % SimCfg::WN;
    const int m0 = blockIdx.x * SimCfg::BM;
    const int split = blockIdx.y;
    const int ntiles = (p.nd + SimCfg::BN - 1) / SimCfg::BN;
    const int t0 = split * p.tiles_per_split, t1 = min(ntiles, t0 + p.tiles_per_split);

    float ts[KMAX];
    int ti[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        ts[j] = -INFINITY;
        ti[j] = 0x7fffffff;
    }
    const int myrow = tid >> 1, half = tid & 1;
    float* tile = reinterpret_cast<float*>(lds);

    for (int t = t0; t < t1; ++t) {
        const int n0 = t * SimCfg::BN;
        f32x4 acc[SimCfg::FM][SimCfg::FN];
        mainloop<SimCfg>(p.Q, p.ldq, p.nq, m0, p.Dm, p.ldd, p.nd, n0, p.D, lds, acc, wave, lane);
        __syncthreads();  // staging buffers are dead; reuse LDS for the score tile
#pragma unroll
        for (int i = 0; i < SimCfg::FM; ++i)
#pragma unroll
            for (int j = 0; j < SimCfg::FN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = wm * SimCfg::TM + i * 16 + 4 * (lane >> 4) + r;
                    const int col = wn * SimCfg::TN + j * 16 + (lane & 15);
                    tile[row * TILE_LD + col] = (n0 + col < p.nd) ? acc[i][j][r] : -INFINITY;
                }
        __syncthreads();
        const float* tr = tile + myrow * TILE_LD + half * 64;
        const int cbase = n0 + half * 64;
        for (int c = 0; c < 64; ++c) topk_insert(ts, ti, tr[c], cbase + c);
        __syncthreads();
    }
    const int row = m0 + myrow;
    if (row < p.nq) {
        const long o = ((long)row * p.nsplit * 2 + split * 2 + half) * p.k;
        for (int j = 0; j < p.k; ++j) {
            p.cand_s[o + j] = ts[j];
            p.cand_i[o + j] = ti[j] == 0x7fffffff ? -1 : ti[j] + p.col_offset;
        }
    }
}

// One wave per row: repeatedly extract the best (score desc, idx asc) candidate.
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ cs, const int* __restrict__ ci,
                                                         int rows, int ncand, int k, int32_t* __restrict__ oi,
                                                         float* __restrict__ os) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float* s = cs + (long)row * ncand;
    const int* ix = ci + (long)row * ncand;
    // each lane keeps its own best-first cursor over a strided slice
    constexpr int PER = 16;
    float vs[PER];
    int vi[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = lane + j * 64;
        const bool ok = c < ncand && ix[c] >= 0;
        vs[j] = ok ? s[c] : -INFINITY;
        vi[j] = ok ? ix[c] : 0x7fffffff;
    }
    for (int out = 0; out < k; ++out) {
        // lane-local best
        float bv = -INFINITY;
        int bi = 0x7fffffff, bj = -1;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const bool better = vs[j] > bv || (vs[j] == bv && vi[j] < bi);
            if (better) {
                bv = vs[j];
                bi = vi[j];
                bj = j;
            }
        }
        float wv = bv;
        int wi = bi;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(wv, o, 64);
            const int oi2 = __shfl_xor(wi, o, 64);
            if (ov > wv || (ov == wv && oi2 < wi)) {
                wv = ov;
                wi = oi2;
            }
        }
        if (lane == 0) {
            oi[(long)row * k + out] = wi == 0x7fffffff ? -1 : wi;
            os[(long)row * k + out] = wv;
        }
        if (bj >= 0 && bi == wi && bv == wv) {
#pragma unroll
            for (int j = 0; j < PER; ++j)
                if (j == bj) {
                    vs[j] = -INFINITY;
                    vi[j] = 0x7fffffff;
                }
        }
    }
}

// Full fp32 score rows through sim_topk_kernel's own main loop: the same MFMA sequence per
// output element, so every score is bit-identical to the one sim_topk ranked. Used for the
// few rows whose top-(k+1) holds an EXACT tie (duplicated images / captions): torch.topk's
// order among tied values (main.py:335,365,375) is re-selected from these rows by
// topk_rows_torch_kernel. 16 lanes store 64 contiguous bytes per row segment.
__global__ __launch_bounds__(SimCfg::NT) void sim_scores_kernel(const bf16* __restrict__ Q, int ldq, int nq,
                                                                const bf16* __restrict__ Dm, int ldd, int nd, int D,
                                                                float* __restrict__ out, long ldo) {
    __shared__ __attribute__((aligned(16))) char lds[SimCfg::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / SimCfg::WN, wn = wave % SimCfg::WN;
    const int m0 = blockIdx.x * SimCfg::BM, n0 = blockIdx.y * SimCfg::BN;
    f32x4 acc[SimCfg::FM][SimCfg::FN];
    mainloop<SimCfg>(Q, ldq, nq, m0, Dm, ldd, nd, n0, D, lds, acc, wave, lane);
#pragma unroll
    for (int i = 0; i < SimCfg::FM; ++i)
#pragma unroll
        for (int j = 0; j < SimCfg::FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * SimCfg::TM + i * 16 + 4 * (lane >> 4) + r;
                const int col = n0 + wn * SimCfg::TN + j * 16 + (lane & 15);
                if (row < nq && col < nd) out[(long)row * ldo + col] = acc[i][j][r];
            }
}

// flags[r] = 1 when the sorted top-k list of row r holds two EXACTLY equal neighbours: only
// then can torch.topk's choice among tied columns differ from the (score desc, column asc)
// order sim_topk produced.
__global__ void tie_rows_kernel(const float* __restrict__ sc, int rows, int k, uint8_t* __restrict__ flags) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const float* s = sc + (long)r * k;
    bool t = false;
    for (int j = 1; j < k; ++j) t |= s[j] == s[j - 1];
    flags[r] = t ? 1 : 0;
}

__global__ void recall_kernel(const int32_t* __restrict__ idx, int rows, int k, const int32_t* __restrict__ tstart,
                              int tcount, int row_offset, const int32_t* __restrict__ kk, int nk,
                              const uint8_t* __restrict__ skip, unsigned long long* __restrict__ hits) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows || (skip && skip[r])) return;
    const int lo = tstart ? tstart[r] : (r + row_offset) * tcount;
    const int hi = lo + tcount;
    int first = k;  // first rank holding a target
    for (int j = 0; j < k; ++j) {
        const int c = idx[(long)r * k + j];
        if (c >= lo && c < hi) {
            first = j;
            break;
        }
    }
    for (int j = 0; j < nk; ++j)
        if (first < min(kk[j], k)) atomicAdd(&hits[j], 1ull);
}

// Row top-k of a materialised fp32 score matrix (the MaxSim scores of the ColPali
// branch; main.py:335,365,375 torch.topk per row). One wave per row: each lane
// scans columns lane, lane+64, ... into a sorted register list (ties keep the
// lower column: a lane scans its columns in increasing order), then k rounds of
// a wave-wide (score desc, column asc) arg-max pop the lanes' list heads.
__global__ __launch_bounds__(256) void topk_rows_kernel(const float* __restrict__ S, int ld, int rows, int cols,
                                                        int k, int col_offset, int32_t* __restrict__ oi,
                                                        float* __restrict__ os) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    float ts[KMAX];
    int ti[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
        ts[j] = -INFINITY;
        ti[j] = 0x7fffffff;
    }
    const float* sr = S + (long)row * ld;
    for (int c = lane; c < cols; c += 64) topk_insert(ts, ti, sr[c], c);
    for (int out = 0; out < k; ++out) {
        float wv = ts[0];
        int wi = ti[0];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(wv, o, 64);
            const int ox = __shfl_xor(wi, o, 64);
            if (ov > wv || (ov == wv && ox < wi)) {
                wv = ov;
                wi = ox;
            }
        }
        if (lane == 0) {
            oi[(long)row * k + out] = wi == 0x7fffffff ? -1 : wi + col_offset;
            os[(long)row * k + out] = wv;
        }
        if (ti[0] == wi && wi != 0x7fffffff) {  // the owner pops its head (column ids are unique)
#pragma unroll
            for (int j = 0; j < KMAX - 1; ++j) {
                ts[j] = ts[j + 1];
                ti[j] = ti[j + 1];
            }
            ts[KMAX - 1] = -INFINITY;
            ti[KMAX - 1] = 0x7fffffff;
        }
    }
}

// ---------------------------------------------------------------------------
// Row top-k in torch.topk's CPU order (main.py:335,365,375 call torch.topk(row, k)
// per row on the CPU). torch's CPU kernel (aten SortingKernel.cpp topk_impl_loop)
// builds (value, column) pairs and, with comp(x, y) = x.value > y.value (NaN first),
// runs libstdc++'s std::partial_sort when k * 64 <= n (heap select over the first k,
// then sort_heap) and otherwise std::nth_element(k - 1) + std::sort of the first k - 1
// (introselect: median-of-3 pivot, unguarded partition, heap-select fallback at
// depth 2 floor(log2 n), insertion sort of <= 3). Exact ties -- the rule with ColPali's
// bf16-quantised MaxSim sums -- therefore come out in that algorithm's order, not by
// column; this kernel replays the same algorithm step for step (oracle:
// oracle/torch_topk.cpp, which calls the libstdc++ algorithms themselves).
//
// k * 64 <= n (every configs[3] row): one wave per row. The heap (k <= 16 pairs)
// lives in LDS; the row streams through in 64-column chunks, and a ballot of
// `value > heap top` picks the only columns heap select can act on (the top only
// grows), which are then replayed in column order. Otherwise (n < 64 k <= 1024):
// nth_element + sort on a copy of the row in the workspace.
struct TPair {
    float v;
    int i;
};
__device__ __forceinline__ bool tcomp(const TPair& x, const TPair& y) {  // torch: largest, NaN first
    return (__builtin_isnan(x.v) && !__builtin_isnan(y.v)) || (x.v > y.v);
}
// libstdc++ std::__adjust_heap + std::__push_heap (bits/stl_heap.h), comp = tcomp
__device__ void heap_adjust(TPair* h, int hole, int len, TPair value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (tcomp(h[second], h[second - 1])) second--;
        h[hole] = h[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        h[hole] = h[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && tcomp(h[parent], value)) {
        h[hole] = h[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    h[hole] = value;
}
__device__ void heap_make(TPair* h, int len) {  // std::__make_heap
    if (len < 2) return;
    for (int parent = (len - 2) / 2;; --parent) {
        heap_adjust(h, parent, len, h[parent]);
        if (parent == 0) return;
    }
}
__device__ void heap_sort(TPair* h, int len) {  // std::__sort_heap
    while (len > 1) {
        --len;
        const TPair value = h[len];
        h[len] = h[0];
        heap_adjust(h, 0, len, value);
    }
}
// std::__heap_select(first, middle, last) on a materialised range
__device__ void heap_select_range(TPair* q, int middle, int last) {
    heap_make(q, middle);
    for (int i = middle; i < last; ++i)
        if (tcomp(q[i], q[0])) {  // std::__pop_heap(first, middle, i)
            const TPair value = q[i];
            q[i] = q[0];
            heap_adjust(q, 0, middle, value);
        }
}
__device__ __forceinline__ void tswap(TPair* a, TPair* b) {
    const TPair t = *a;
    *a = *b;
    *b = t;
}
__device__ void insertion_sort(TPair* q, int first, int last) {  // std::__insertion_sort
    if (first == last) return;
    for (int i = first + 1; i < last; ++i) {
        const TPair val = q[i];
        if (tcomp(val, q[first])) {
            for (int j = i; j > first; --j) q[j] = q[j - 1];  // move_backward
            q[first] = val;
        } else {  // std::__unguarded_linear_insert
            int last_ = i, next = i - 1;
            while (tcomp(val, q[next])) {
                q[last_] = q[next];
                last_ = next;
                --next;
            }
            q[last_] = val;
        }
    }
}
__device__ void move_median_to_first(TPair* q, int result, int a, int b, int c) {
    if (tcomp(q[a], q[b])) {
        if (tcomp(q[b], q[c])) tswap(q + result, q + b);
        else if (tcomp(q[a], q[c])) tswap(q + result, q + c);
        else tswap(q + result, q + a);
    } else if (tcomp(q[a], q[c])) tswap(q + result, q + a);
    else if (tcomp(q[b], q[c])) tswap(q + result, q + c);
    else tswap(q + result, q + b);
}
__device__ int unguarded_partition(TPair* q, int first, int last, int pivot) {
    while (true) {
        while (tcomp(q[first], q[pivot])) ++first;
        --last;
        while (tcomp(q[pivot], q[last])) --last;
        if (!(first < last)) return first;
        tswap(q + first, q + last);
        ++first;
    }
}
__device__ void nth_element_torch(TPair* q, int nth, int n) {  // std::nth_element -> std::__introselect
    if (n == 0 || nth == n) return;
    int first = 0, last = n;
    int depth = 2 * (31 - __builtin_clz(n));  // std::__lg(n) * 2
    while (last - first > 3) {
        if (depth == 0) {
            heap_select_range(q + first, nth + 1 - first, last - first);
            tswap(q + first, q + nth);
            return;
        }
        --depth;
        const int mid = first + (last - first) / 2;
        move_median_to_first(q, first, first + 1, mid, last - 1);
        const int cut = unguarded_partition(q, first + 1, last, first);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort(q, first, last);
}

// Every lane of the wave runs the (uniform) algorithm itself on the shared LDS heap /
// workspace row -- the same reads and writes of the same values in every lane -- so no
// lane ever depends on another lane's memory writes.
__global__ __launch_bounds__(256) void topk_rows_torch_kernel(const float* __restrict__ S, int ld, int rows, int cols,
                                                              int k, int col_offset, int32_t* __restrict__ oi,
                                                              float* __restrict__ os, TPair* __restrict__ ws) {
    __shared__ TPair heaps[4][KMAX];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wv;
    if (row >= rows) return;  // wave-uniform
    const float* sr = S + (long)row * ld;
    TPair* q;
    if ((long)k * 64 <= cols) {  // std::partial_sort(q, q + k, q + n): heap select + sort_heap
        q = heaps[wv];
        for (int j = 0; j < k; ++j) q[j] = TPair{sr[j], j};
        heap_make(q, k);
        for (int c0 = k; c0 < cols; c0 += 64) {
            const int c = c0 + lane;
            const float v = c < cols ? sr[c] : 0.f;
            const TPair top = q[0];
            unsigned long long m = __ballot(c < cols && tcomp(TPair{v, c}, top));
            while (m) {  // candidates in column order (the top only grows: no other column acts)
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                const float vb = __shfl(v, b, 64);
                if (tcomp(TPair{vb, 0}, q[0])) heap_adjust(q, 0, k, TPair{vb, c0 + b});  // __pop_heap(first, middle, i)
            }
        }
        heap_sort(q, k);
    } else {  // std::nth_element(q, q + k - 1, q + n) + std::sort(q, q + k - 1)
        q = ws + (long)row * cols;
        for (int c = 0; c < cols; ++c) q[c] = TPair{sr[c], c};
        nth_element_torch(q, k - 1, cols);
        insertion_sort(q, 0, k - 1);  // std::sort of <= 15 elements = its final insertion sort
    }
    if (lane < k) {
        oi[(long)row * k + lane] = q[lane].i + col_offset;
        os[(long)row * k + lane] = q[lane].v;
    }
}

// Winoground 2x2 scoring (run_winoground, run_benchmark_grand_slam_v28_publication_ready.py:
// 413-461): per example s[t][i] = bf16( <text_t, image_i> ) — torch.matmul on the bf16
// (normalised) embeddings, fp32 accumulation, one rounding — then the strict comparisons
// text: s00>s01 && s11>s10, image: s00>s10 && s11>s01, group: both. One wave per example.
__global__ __launch_bounds__(256) void winoground_kernel(const bf16* __restrict__ T, const bf16* __restrict__ I,
                                                         int n, int D, float* __restrict__ scores,
                                                         unsigned long long* __restrict__ counts) {
    const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= n) return;
    const bf16* t0 = T + (long)e * 2 * D;
    const bf16* i0 = I + (long)e * 2 * D;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = lane; c < D / 8; c += 64) {
        const u16x8 a0 = *reinterpret_cast<const u16x8*>(t0 + c * 8);
        const u16x8 a1 = *reinterpret_cast<const u16x8*>(t0 + D + c * 8);
        const u16x8 b0 = *reinterpret_cast<const u16x8*>(i0 + c * 8);
        const u16x8 b1 = *reinterpret_cast<const u16x8*>(i0 + D + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            acc[0] += bits2f(a0[j]) * bits2f(b0[j]);
            acc[1] += bits2f(a0[j]) * bits2f(b1[j]);
            acc[2] += bits2f(a1[j]) * bits2f(b0[j]);
            acc[3] += bits2f(a1[j]) * bits2f(b1[j]);
        }
    }
    float s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = bf2f(f2bf(wave_sum(acc[j])));
    if (lane == 0) {
        for (int j = 0; j < 4; ++j) scores[(long)e * 4 + j] = s[j];
        const bool txt = s[0] > s[1] && s[3] > s[2];
        const bool img = s[0] > s[2] && s[3] > s[1];
        if (txt) atomicAdd(&counts[0], 1ull);
        if (img) atomicAdd(&counts[1], 1ull);
        if (txt && img) atomicAdd(&counts[2], 1ull);
    }
}

// Bootstrap resampling (main.py:586-624): the score matrices of one resample are
// index gathers of the full matrices: out[b][i][p] = S[rows[b][i]][g*cols[b][p/g] + p%g]
// (T2I: g = 1; I2T: g = 5 captions per sampled image, compute_similarity_scores over
// all_txt[sampled_i2t_cap_indices]; I2T-Sym: the transposed T2I matrix, g = 1).
// One block per output row; 16-B coalesced stores; the column gather reads S[row]
// (20 KB / 100 KB rows, L2/MALL-resident across the rows that share it).
__global__ __launch_bounds__(256) void gather_scores_kernel(const float* __restrict__ S, long ld,
                                                            const int32_t* __restrict__ rows,
                                                            const int32_t* __restrict__ cols, int R, int C, int g,
                                                            float* __restrict__ out) {
    const long orow = blockIdx.x;  // b*R + i
    const int b = orow / R;
    const float* src = S + (long)rows[orow] * ld;
    const int32_t* cb = cols + (long)b * C;
    const int W = C * g;
    float* dst = out + orow * W;
    for (int p0 = threadIdx.x * 4; p0 < W; p0 += 256 * 4) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int p = p0 + e;
            v[e] = p < W ? src[(long)g * cb[p / g] + p % g] : 0.f;
        }
        if (p0 + 3 < W && (W & 3) == 0) {
            *reinterpret_cast<float4*>(dst + p0) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            for (int e = 0; e < 4; ++e)
                if (p0 + e < W) dst[p0 + e] = v[e];
        }
    }
}

// Recall hits per group of R rows (one bootstrap resample per group): row r of group
// b targets columns [(r % R) * tc, (r % R) * tc + tc); hits[b][j] += row hit within kk[j].
__global__ void recall_groups_kernel(const int32_t* __restrict__ idx, int rows, int k, int R, int tc,
                                     const int32_t* __restrict__ kk, int nk, unsigned long long* __restrict__ hits) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int lo = (r % R) * tc, hi = lo + tc;
    int first = k;
    for (int j = 0; j < k; ++j) {
        const int c = idx[(long)r * k + j];
        if (c >= lo && c < hi) {
            first = j;
            break;
        }
    }
    for (int j = 0; j < nk; ++j)
        if (first < min(kk[j], k)) atomicAdd(&hits[(long)(r / R) * nk + j], 1ull);
}

size_t sim_splits(int nq, int nd, int k, int* tiles_per_split) {
    const int nqt = (nq + 127) / 128, ntiles = (nd + 127) / 128;
    // aim for >= 1024 workgroups, >= 4 tiles per split, and a candidate list
    // (nsplit * 2 halves * k) the one-wave merge can hold (<= 1024)
    int nsplit = (1024 + nqt - 1) / nqt;
    nsplit = min(nsplit, max(1, ntiles / 4));
    nsplit = min(nsplit, 512 / k);
    nsplit = max(1, min(nsplit, ntiles));
    *tiles_per_split = (ntiles + nsplit - 1) / nsplit;
    nsplit = (ntiles + *tiles_per_split - 1) / *tiles_per_split;
    return (size_t)nsplit;
}

}  // namespace

extern "C" size_t mme_sim_topk_workspace_bytes(int nq, int nd, int k) {
    int tps;
    const size_t nsplit = sim_splits(nq, nd, k, &tps);
    return (size_t)nq * nsplit * 2 * k * (sizeof(float) + sizeof(int)) + 256;
}

extern "C" int mme_sim_topk(const void* Q, int ldq, const void* Db, int ldd, int nq, int nd, int D, int k,
                            int col_offset, int32_t* out_idx, float* out_score, void* workspace, size_t ws_bytes,
                            void* stream) {
    MME_REQUIRE(Q && Db && out_idx && out_score && workspace, "mme_sim_topk: null pointer");
    MME_REQUIRE(nq >= 0 && nd > 0 && D > 0 && D % 64 == 0, "mme_sim_topk: D=%d must be a multiple of 64", D);
    MME_REQUIRE(k >= 1 && k <= KMAX && k <= nd, "mme_sim_topk: k=%d out of range (<= %d, <= nd)", k, KMAX);
    MME_REQUIRE(ldq % 8 == 0 && ldd % 8 == 0 && ldq >= D && ldd >= D, "mme_sim_topk: bad leading dims");
    MME_REQUIRE(ws_bytes >= mme_sim_topk_workspace_bytes(nq, nd, k), "mme_sim_topk: workspace too small");
    if (nq == 0) return MME_OK;
    int tps;
    const int nsplit = (int)sim_splits(nq, nd, k, &tps);
    float* cs = (float*)workspace;
    int* ci = (int*)((char*)workspace + (size_t)nq * nsplit * 2 * k * sizeof(float));
    SimArgs a{(const bf16*)Q, (const bf16*)Db, ldq, ldd, nq, nd, D, k, col_offset, tps, nsplit, cs, ci};
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(sim_topk_kernel, dim3((nq + 127) / 128, nsplit), dim3(SimCfg::NT), 0, s, a);
    int rc = mme_check_launch("mme_sim_topk");
    if (rc) return rc;
    return mme_topk_merge(ci, cs, nq, nsplit * 2, k, out_idx, out_score, stream);
}

extern "C" int mme_topk_merge(const int32_t* in_idx, const float* in_score, int rows, int parts, int k,
                              int32_t* out_idx, float* out_score, void* stream) {
    MME_REQUIRE(in_idx && in_score && out_idx && out_score, "mme_topk_merge: null pointer");
    MME_REQUIRE(rows >= 0 && parts >= 1 && k >= 1 && (long)parts * k <= 64 * 16,
                "mme_topk_merge: parts*k=%d exceeds 1024", parts * k);
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(topk_merge_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), in_score, in_idx,
                       rows, parts * k, k, out_idx, out_score);
    return mme_check_launch("mme_topk_merge");
}

extern "C" int mme_topk_rows(const float* scores, int ld, int rows, int cols, int k, int col_offset,
                             int32_t* out_idx, float* out_score, void* stream) {
    MME_REQUIRE(scores && out_idx && out_score, "mme_topk_rows: null pointer");
    MME_REQUIRE(rows >= 0 && cols >= 1 && ld >= cols, "mme_topk_rows: bad shape");
    MME_REQUIRE(k >= 1 && k <= KMAX && k <= cols, "mme_topk_rows: k=%d out of range (<= %d, <= cols)", k, KMAX);
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(topk_rows_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), scores, ld, rows, cols,
                       k, col_offset, out_idx, out_score);
    return mme_check_launch("mme_topk_rows");
}

extern "C" size_t mme_topk_rows_torch_workspace_bytes(int rows, int cols, int k) {
    return ((long)k * 64 <= cols) ? 0 : (size_t)rows * cols * sizeof(TPair);
}

extern "C" int mme_topk_rows_torch(const float* scores, int ld, int rows, int cols, int k, int col_offset,
                                   int32_t* out_idx, float* out_score, void* workspace, size_t ws_bytes,
                                   void* stream) {
    MME_REQUIRE(scores && out_idx && out_score, "mme_topk_rows_torch: null pointer");
    MME_REQUIRE(rows >= 0 && cols >= 1 && ld >= cols, "mme_topk_rows_torch: bad shape");
    MME_REQUIRE(k >= 1 && k <= KMAX && k <= cols, "mme_topk_rows_torch: k=%d out of range (<= %d, <= cols)", k, KMAX);
    const size_t need = mme_topk_rows_torch_workspace_bytes(rows, cols, k);
    MME_REQUIRE(ws_bytes >= need && (need == 0 || workspace), "mme_topk_rows_torch: workspace %zu < %zu bytes",
                ws_bytes, need);
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(topk_rows_torch_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), scores, ld, rows,
                       cols, k, col_offset, out_idx, out_score, reinterpret_cast<TPair*>(workspace));
    return mme_check_launch("mme_topk_rows_torch");
}

extern "C" int mme_gather_scores(const float* S, long ld, const int32_t* rows, const int32_t* cols, int B, int R,
                                 int C, int g, float* out, void* stream) {
    MME_REQUIRE(S && rows && cols && out, "mme_gather_scores: null pointer");
    MME_REQUIRE(B >= 0 && R >= 0 && C > 0 && g >= 1 && ld > 0, "mme_gather_scores: bad shape");
    MME_REQUIRE((long)B * R < (1L << 31), "mme_gather_scores: too many output rows");
    if (B == 0 || R == 0) return MME_OK;
    hipLaunchKernelGGL(gather_scores_kernel, dim3(B * R), dim3(256), 0, as_stream(stream), S, ld, rows, cols, R, C, g,
                       out);
    return mme_check_launch("mme_gather_scores");
}

extern "C" int mme_recall_hits_groups(const int32_t* topk_idx, int rows, int k, int R, int tgt_count, const int32_t* kk,
                                      int nk, int64_t* hits, void* stream) {
    MME_REQUIRE(topk_idx && kk && hits, "mme_recall_hits_groups: null pointer");
    MME_REQUIRE(rows >= 0 && k >= 1 && R >= 1 && tgt_count >= 1 && nk >= 1, "mme_recall_hits_groups: bad args");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(recall_groups_kernel, dim3(cdiv(rows, 256)), dim3(256), 0, as_stream(stream), topk_idx, rows, k,
                       R, tgt_count, kk, nk, (unsigned long long*)hits);
    return mme_check_launch("mme_recall_hits_groups");
}

extern "C" int mme_winoground(const void* text, const void* image, int n, int D, float* scores, int64_t* counts,
                              void* stream) {
    MME_REQUIRE(text && image && scores && counts, "mme_winoground: null pointer");
    MME_REQUIRE(n >= 0 && D > 0 && D % 8 == 0, "mme_winoground: D=%d must be a multiple of 8", D);
    if (n == 0) return MME_OK;
    hipLaunchKernelGGL(winoground_kernel, dim3(cdiv(n, 4)), dim3(256), 0, as_stream(stream), (const bf16*)text,
                       (const bf16*)image, n, D, scores, (unsigned long long*)counts);
    return mme_check_launch("mme_winoground");
}

extern "C" int mme_recall_hits(const int32_t* topk_idx, int rows, int k, const int32_t* tgt_start, int tgt_count,
                               int row_offset, const int32_t* kk, int nk, const uint8_t* skip, int64_t* hits,
                               void* stream) {
    MME_REQUIRE(topk_idx && kk && hits, "mme_recall_hits: null pointer");
    MME_REQUIRE(rows >= 0 && k >= 1 && tgt_count >= 1 && nk >= 1, "mme_recall_hits: bad args");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(recall_kernel, dim3(cdiv(rows, 256)), dim3(256), 0, as_stream(stream), topk_idx, rows, k,
                       tgt_start, tgt_count, row_offset, kk, nk, skip, (unsigned long long*)hits);
    return mme_check_launch("mme_recall_hits");
}

extern "C" int mme_sim_scores(const void* Q, int ldq, const void* Db, int ldd, int nq, int nd, int D, float* out,
                              long ldo, void* stream) {
    MME_REQUIRE(Q && Db && out, "mme_sim_scores: null pointer");
    MME_REQUIRE(nq >= 0 && nd > 0 && D > 0 && D % 64 == 0, "mme_sim_scores: D=%d must be a multiple of 64", D);
    MME_REQUIRE(ldq % 8 == 0 && ldd % 8 == 0 && ldq >= D && ldd >= D && ldo >= nd, "mme_sim_scores: bad leading dims");
    MME_REQUIRE(cdiv(nd, SimCfg::BN) <= 65535, "mme_sim_scores: nd=%d too large", nd);
    if (nq == 0) return MME_OK;
    hipLaunchKernelGGL(sim_scores_kernel, dim3(cdiv(nq, SimCfg::BM), cdiv(nd, SimCfg::BN)), dim3(SimCfg::NT), 0,
                       as_stream(stream), (const bf16*)Q, ldq, nq, (const bf16*)Db, ldd, nd, D, out, ldo);
    return mme_check_launch("mme_sim_scores");
}

extern "C" int mme_tie_rows(const float* scores, int rows, int k, uint8_t* flags, void* stream) {
    MME_REQUIRE(scores && flags, "mme_tie_rows: null pointer");
    MME_REQUIRE(rows >= 0 && k >= 1, "mme_tie_rows: bad args");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(tie_rows_kernel, dim3(cdiv(rows, 256)), dim3(256), 0, as_stream(stream), scores, rows, k, flags);
    return mme_check_launch("mme_tie_rows");
}
