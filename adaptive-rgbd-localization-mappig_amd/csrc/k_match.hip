// Matching kernels for gfx950.
//
//   k_knn2        cv::BFMatcher(NORM_HAMMING).knnMatch(k=2)   Features/matcher.cpp:60 (App. A.6)
//   k_pair_match  per frame pair: UpdateLastFrame VO landmarks (tracking.cpp:146-190),
//                 ratio test + landmark bookkeeping (matcher.cpp:62-85),
//                 Ransac good-match filter + std::sort (ransac.cpp:175-199)
//   k_latch       Ransac::DepthCovariance first-call latch (ransac.cpp:416-421)
#include <type_traits>

#include "odo_device.h"
#include "odo_internal.h"

namespace odo {

// ============================================================ kNN-2 Hamming
// One query per lane (256-bit descriptor in 8 VGPRs), train descriptors staged
// through LDS in tiles and read as wave-uniform broadcasts. The top-2 is kept
// as packed keys (dist<<20 | trainIdx): the BFMatcher insertion rule (ties keep
// the lower train index, equal-to-second does not replace) is exactly "the two
// smallest (dist, idx) pairs", so min/max updates reproduce it.
#ifndef KNN_Q
#define KNN_Q 256  // queries (threads) per workgroup
#endif
#define KNN_T 256

ODO_INLINE uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
// (dist << 20) | train index, the index wave-uniform (an SGPR operand)
ODO_INLINE uint32_t key_of(uint32_t d, uint32_t idx) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, 20, %2" : "=v"(r) : "v"(d), "s"(idx));
    return r;
}
ODO_INLINE uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

#ifndef KNN_QPL
#define KNN_QPL 1  // queries per lane (more independent popcount chains per wave)
#endif
#define KNN_TH (KNN_Q / KNN_QPL)      // threads per workgroup
#define KNN_PF (2 * KNN_T / KNN_TH)   // uint4 of a staged train chunk per thread
#define KNN_MAXP 1024                 // pairs per launch (the item prefix lives in LDS)
__global__ void __launch_bounds__(KNN_TH) k_knn2(const uint8_t* __restrict__ qdesc, const int* __restrict__ qn,
                                                 size_t q_stride, const uint8_t* __restrict__ tdesc,
                                                 const int* __restrict__ tn, size_t t_stride,
                                                 int2* __restrict__ out_idx, int2* __restrict__ out_dist,
                                                 size_t out_stride, const int32_t* __restrict__ qlist,
                                                 const int* __restrict__ qcnt, size_t ql_stride,
                                                 size_t split_stride, int npairs, int qblocks, int nsplit) {
#ifndef ODO_KNN_PRIO
#define ODO_KNN_PRIO 2  // co-runs with the previous batch's PnP: issue first (+0.07 roofline, same step time)
#endif
    __builtin_amdgcn_s_setprio(ODO_KNN_PRIO);
    __shared__ uint4 tile[KNN_T * 2];
    // A fixed grid (one round of resident workgroups) shares out the active
    // items (pair, block of KNN_Q queries, train split) in contiguous equal
    // runs: the items of one query block are consecutive, so a run reloads
    // its queries and writes its top-2 only when the block changes (the
    // block's other split slots it covered get an empty entry; the consumer
    // merges the splits). The next train chunk is loaded into registers while
    // the current chunk is compared.
    __shared__ int s_pre[KNN_MAXP + 1];
    const int tid = threadIdx.x;
    // exclusive prefix of the pairs' active item counts
    for (int i = tid; i < npairs; i += KNN_TH) {
        const int nq = qlist ? qcnt[i] : qn[i];
        s_pre[i + 1] = ((nq + KNN_Q - 1) / KNN_Q) * nsplit;
    }
    if (tid == 0) s_pre[0] = 0;
    __syncthreads();
    if (tid == 0)
        for (int i = 1; i <= npairs; i++) s_pre[i] += s_pre[i - 1];
    __syncthreads();
    const int nact = s_pre[npairs];
    const int g0 = (int)((long)nact * blockIdx.x / gridDim.x), g1 = (int)((long)nact * (blockIdx.x + 1) / gridDim.x);
    struct Item {
        int p, qbk, h, tb, te;
    };
    auto decode = [&](int g) -> Item {
        int lo = 0, hi = npairs;  // last pair with s_pre[p] <= g
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_pre[mid] <= g) lo = mid; else hi = mid;
        }
        Item I;
        I.p = lo;
        const int local = g - s_pre[lo];
        I.qbk = local / nsplit;
        I.h = local - I.qbk * nsplit;
        const int nt = tn[I.p];
        I.tb = (int)((long)nt * I.h / nsplit);
        I.te = (int)((long)nt * (I.h + 1) / nsplit);
        return I;
    };
    uint4 r[KNN_PF];  // prefetched train chunk
#pragma unroll
    for (int k = 0; k < KNN_PF; k++) r[k] = make_uint4(0, 0, 0, 0);
    auto load_chunk = [&](int p, int t0, int te) {
        const int cnt = min(KNN_T, te - t0);
        const uint4* src = reinterpret_cast<const uint4*>(tdesc + (size_t)p * t_stride + (size_t)t0 * 32);
#pragma unroll
        for (int k = 0; k < KNN_PF; k++)
            if (tid + k * KNN_TH < 2 * cnt) r[k] = src[tid + k * KNN_TH];
    };
    int cur_p = -1, cur_qbk = -1, h_first = 0, h_last = 0;
    int qi[KNN_QPL];
    uint32_t q[KNN_QPL][8], k0[KNN_QPL], k1[KNN_QPL];
    auto flush = [&]() {  // the run's top-2 into split slot h_first, empties into the others it covered
        if (cur_p < 0) return;
#pragma unroll
        for (int s = 0; s < KNN_QPL; s++) {
            if (qi[s] < 0) continue;
            int2 I, D;
            I.x = k0[s] == 0xFFFFFFFFu ? -1 : (int)(k0[s] & 0xFFFFF);
            D.x = k0[s] == 0xFFFFFFFFu ? 0x7FFFFFFF : (int)(k0[s] >> 20);
            I.y = k1[s] == 0xFFFFFFFFu ? -1 : (int)(k1[s] & 0xFFFFF);
            D.y = k1[s] == 0xFFFFFFFFu ? 0x7FFFFFFF : (int)(k1[s] >> 20);
            const size_t o = (size_t)cur_p * out_stride + qi[s];
            out_idx[(size_t)h_first * split_stride + o] = I;
            out_dist[(size_t)h_first * split_stride + o] = D;
            for (int hh = h_first + 1; hh <= h_last; hh++) {
                out_idx[(size_t)hh * split_stride + o] = make_int2(-1, -1);
                out_dist[(size_t)hh * split_stride + o] = make_int2(0x7FFFFFFF, 0x7FFFFFFF);
            }
        }
    };
    if (g0 < g1) {
        const Item I = decode(g0);
        if (I.te > I.tb) load_chunk(I.p, I.tb, I.te);
    }
    for (int g = g0; g < g1; g++) {
        const Item I = decode(g);
        if (I.p != cur_p || I.qbk != cur_qbk) {
            flush();
            cur_p = I.p;
            cur_qbk = I.qbk;
            h_first = I.h;
            const int nq = qlist ? qcnt[I.p] : qn[I.p];
            const uint8_t* Q = qdesc + (size_t)I.p * q_stride;
#pragma unroll
            for (int s = 0; s < KNN_QPL; s++) {
                const int qpos = I.qbk * KNN_Q + s * KNN_TH + tid;
                qi[s] = qpos < nq ? (qlist ? qlist[(size_t)I.p * ql_stride + qpos] : qpos) : -1;
                uint4 qa = make_uint4(0, 0, 0, 0), qb = make_uint4(0, 0, 0, 0);
                if (qi[s] >= 0) {
                    qa = reinterpret_cast<const uint4*>(Q + (size_t)qi[s] * 32)[0];
                    qb = reinterpret_cast<const uint4*>(Q + (size_t)qi[s] * 32)[1];
                }
                q[s][0] = qa.x, q[s][1] = qa.y, q[s][2] = qa.z, q[s][3] = qa.w;
                q[s][4] = qb.x, q[s][5] = qb.y, q[s][6] = qb.z, q[s][7] = qb.w;
                k0[s] = 0xFFFFFFFFu;
                k1[s] = 0xFFFFFFFFu;
            }
        }
        h_last = I.h;
        const bool more = g + 1 < g1;
        if (I.te <= I.tb && more) {  // empty split: the next item's first chunk now
            const Item N = decode(g + 1);
            if (N.te > N.tb) load_chunk(N.p, N.tb, N.te);
        }
        for (int t0 = I.tb; t0 < I.te; t0 += KNN_T) {
            const int tcount = min(KNN_T, I.te - t0);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < KNN_PF; k++) tile[tid + k * KNN_TH] = r[k];
            __syncthreads();
            if (t0 + KNN_T < I.te) {
                load_chunk(I.p, t0 + KNN_T, I.te);
            } else if (more) {
                const Item N = decode(g + 1);
                if (N.te > N.tb) load_chunk(N.p, N.tb, N.te);
            }
            // 8 xor + 8 accumulating bcnt, then key and the top-2 update as
            // min + med3 (k0 <= k1 always holds): 19 VALU per comparison; four
            // train descriptors interleaved so the bcnt chains overlap
            int j = 0;
            for (; j + 4 <= tcount; j += 4) {
                uint32_t d[KNN_QPL][4], t[4][8];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint4 ta = tile[2 * (j + u)], tb2 = tile[2 * (j + u) + 1];
                    t[u][0] = ta.x, t[u][1] = ta.y, t[u][2] = ta.z, t[u][3] = ta.w;
                    t[u][4] = tb2.x, t[u][5] = tb2.y, t[u][6] = tb2.z, t[u][7] = tb2.w;
#pragma unroll
                    for (int s = 0; s < KNN_QPL; s++) d[s][u] = 0u;
                }
#pragma unroll
                for (int w = 0; w < 8; w++)
#pragma unroll
                    for (int s = 0; s < KNN_QPL; s++)
#pragma unroll
                        for (int u = 0; u < 4; u++) d[s][u] = bcnt_acc(q[s][w] ^ t[u][w], d[s][u]);
#pragma unroll
                for (int s = 0; s < KNN_QPL; s++)
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const uint32_t key = key_of(d[s][u], (uint32_t)(t0 + j + u));
                        k1[s] = med3_u32(k0[s], k1[s], key);
                        k0[s] = min(k0[s], key);
                    }
            }
            for (; j < tcount; j++) {
                const uint4 ta = tile[2 * j], tb2 = tile[2 * j + 1];
                const uint32_t tw[8] = {ta.x, ta.y, ta.z, ta.w, tb2.x, tb2.y, tb2.z, tb2.w};
#pragma unroll
                for (int s = 0; s < KNN_QPL; s++) {
                    uint32_t d = 0u;
#pragma unroll
                    for (int w = 0; w < 8; w++) d = bcnt_acc(q[s][w] ^ tw[w], d);
                    const uint32_t key = (d << 20) | (uint32_t)(t0 + j);
                    k1[s] = med3_u32(k0[s], k1[s], key);
                    k0[s] = min(k0[s], key);
                }
            }
        }
    }
    flush();
}

// ============================================================ kNN-2 Hamming on the matrix cores
// Exact integer reformulation of the same comparison. With s(b) = +1 / -1 for a
// descriptor bit 0 / 1, the dot product of two descriptors' sign vectors is
// 256 - 2H (H = Hamming distance). k_knn2_mx feeds the train signs scaled by +64
// and the query signs scaled by -64 to v_mfma_i32_16x16x64_i8, so a 256-bit
// comparison is four k-steps whose i32 sum is -4096 (256 - 2H) = 8192 H - 2^20.
// The accumulator starts at the train index, so the MFMA result is already the
// packed key 8192 H + idx - 2^20 (idx < 8192), ordered exactly as (H, idx): the
// BFMatcher top-2 is min + med3 on signed keys, two VALU ops per comparison
// instead of k_knn2's 19.
//
// Layout: a workgroup item is (pair, block of 256 queries); each of its 4 waves
// holds 64 queries as the MFMA B operand (4 query tiles x 4 k-steps x 16 signed
// bytes per lane = 64 VGPRs, expanded once per item). Trains stream through LDS
// in chunks of 64: each thread expands 4 of a chunk's 1024 (train, 16-bit unit)
// pieces into 16 signed bytes (double-buffered, one barrier per chunk); the
// 16-byte pieces of a train are XOR-swizzled by the train index so the A-operand
// ds_read_b128 of 16 consecutive trains hits distinct banks. The output
// D[train][query] puts 4 trains of one query in each lane; the 4 lane groups
// holding a query are merged with two xor-shuffles at the end of the item.
#define KMX_Q 256       // queries per item (4 waves x 64)
#define KMX_T 64        // trains per LDS chunk
#define KMX_EMPTY 0x7FFFFFFF
#define KMX_BIG 0x3FFFFFFF  // accumulator start of a train slot past the end (never a top-2 key)
typedef int kmx_v4i __attribute__((ext_vector_type(4)));

// 16 descriptor bits -> 16 bytes: bit 0 -> +64 (0x40), bit 1 -> -64 (0xC0)
ODO_INLINE kmx_v4i kmx_expand16(uint32_t h) {
    kmx_v4i r;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t nib = __builtin_amdgcn_ubfe(h, 4 * j, 4);
        // asm: left to itself the compiler folds the << 7 into the constant
        // (v_mul_lo_u32, quarter rate) or splits the shift-or in two
        uint32_t m, b;
        asm("v_mul_u32_u24 %0, %1, %2" : "=v"(m) : "v"(nib), "v"(0x204081u));
        asm("v_lshl_or_b32 %0, %1, 7, %2" : "=v"(b) : "v"(m & 0x01010101u), "s"(0x40404040u));  // bit i -> byte i
        r[j] = (int)b;
    }
    return r;
}
// v_med3_i32 by pattern (not inline asm: its operands come straight from MFMA
// results, and the hazard recognizer inserts the MFMA-to-VALU wait states only
// for instructions it sees)
ODO_INLINE int med3_i32(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

#ifdef ODO_TUNING  // retired int8 form (A/B only: the tuning build)
// (256, 3): 168 VGPRs, three workgroups per CU (measured 137 us vs 144 us at two)
__global__ void __launch_bounds__(256, 3) k_knn2_mx(const uint8_t* __restrict__ qdesc, const int* __restrict__ qn,
                                                 size_t q_stride, const uint8_t* __restrict__ tdesc,
                                                 const int* __restrict__ tn, size_t t_stride,
                                                 int2* __restrict__ out_idx, int2* __restrict__ out_dist,
                                                 size_t out_stride, const int32_t* __restrict__ qlist,
                                                 const int* __restrict__ qcnt, size_t ql_stride, int npairs) {
    __builtin_amdgcn_s_setprio(ODO_KNN_PRIO);
    __shared__ __attribute__((aligned(16))) uint8_t s_tr[2][KMX_T * 256];
    __shared__ int s_pre[KNN_MAXP + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, col = lane & 15;
    for (int i = tid; i < npairs; i += 256) {
        const int nq = qlist ? qcnt[i] : qn[i];
        s_pre[i + 1] = (nq + KMX_Q - 1) / KMX_Q;
    }
    if (tid == 0) s_pre[0] = 0;
    __syncthreads();
    if (tid == 0)
        for (int i = 1; i <= npairs; i++) s_pre[i] += s_pre[i - 1];
    __syncthreads();
    const int nact = s_pre[npairs];
    // staging role of this thread: train st_t of a chunk, 16-bit units 4 st_q .. 4 st_q + 3
    const int st_t = tid >> 2, st_q = tid & 3;
    for (int g = blockIdx.x; g < nact; g += gridDim.x) {
        int lo = 0, hi = npairs;  // last pair with s_pre[p] <= g
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_pre[mid] <= g) lo = mid; else hi = mid;
        }
        const int p = lo, qb = g - s_pre[p];
        const int nq = qlist ? qcnt[p] : qn[p];
        const int nt = tn[p];
        const uint8_t* Q = qdesc + (size_t)p * q_stride;
        const uint8_t* T = tdesc + (size_t)p * t_stride;
        const int qbase = qb * KMX_Q + wave * 64;
        // ---- B operand: this wave's 64 queries, sign bytes scaled by -64 (the
        // complemented bits expanded as trains are)
        kmx_v4i B[4][4];
#pragma unroll
        for (int qt = 0; qt < 4; qt++) {
            const int qpos = qbase + qt * 16 + col;
            uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
            if (qpos < nq) {
                const int qi = qlist ? qlist[(size_t)p * ql_stride + qpos] : qpos;
                a = reinterpret_cast<const uint4*>(Q + (size_t)qi * 32)[0];
                b = reinterpret_cast<const uint4*>(Q + (size_t)qi * 32)[1];
            }
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int u = 4 * c + grp;  // 16-bit unit of k-step c, lane group grp
                uint32_t h = 0;
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (k == u) h = (k & 1) ? (w[k >> 1] >> 16) : (w[k >> 1] & 0xFFFFu);
                B[qt][c] = kmx_expand16(~h & 0xFFFFu);
            }
        }
        int k0[4], k1[4];
#pragma unroll
        for (int qt = 0; qt < 4; qt++) k0[qt] = k1[qt] = KMX_EMPTY;
        const int nch = (nt + KMX_T - 1) / KMX_T;
        uint2 pf = make_uint2(0, 0);
        auto fetch = [&](int ch) {
            const int t = ch * KMX_T + st_t;
            pf = t < nt ? *reinterpret_cast<const uint2*>(T + (size_t)t * 32 + 8 * st_q) : make_uint2(0, 0);
        };
        auto stage = [&](int buf) {
            uint8_t* dst = s_tr[buf] + st_t * 256;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t h = (k < 2 ? pf.x : pf.y) >> (16 * (k & 1)) & 0xFFFFu;
                const int u = 4 * st_q + k;
                *reinterpret_cast<kmx_v4i*>(dst + ((u ^ (st_t & 15)) << 4)) = kmx_expand16(h);
            }
        };
        __syncthreads();  // the previous item's last chunk is no longer read
        if (nch > 0) {
            fetch(0);
            stage(0);
        }
        __syncthreads();
        const bool live = qbase < nq;  // wave-uniform: this wave holds queries
        // One chunk of 64 trains against the wave's 64 queries: 4 tiles of 16
        // trains, each 4 k-steps x 4 query tiles = 16 MFMAs. The 4 A reads of
        // tile tt + 1 are issued before tile tt's MFMAs, so the LDS latency
        // hides behind them. A full chunk starts each accumulator at its train
        // index; only the last, partial chunk selects KMX_BIG for the pad rows.
        auto chunk = [&](const uint8_t* src, int cbase, auto full_tag) {
            constexpr bool full = decltype(full_tag)::value;
            kmx_v4i A[2][4];
#pragma unroll
            for (int c = 0; c < 4; c++)
                A[0][c] = *reinterpret_cast<const kmx_v4i*>(src + col * 256 + (((4 * c + grp) ^ col) << 4));
#pragma unroll
            for (int tt = 0; tt < KMX_T / 16; tt++) {
                const int cur = tt & 1;
                if (tt + 1 < KMX_T / 16) {
                    const int r = (tt + 1) * 16 + col;  // train row of this lane's next A operand
#pragma unroll
                    for (int c = 0; c < 4; c++)
                        A[cur ^ 1][c] = *reinterpret_cast<const kmx_v4i*>(src + r * 256 + (((4 * c + grp) ^ col) << 4));
                }
                kmx_v4i C;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int idx = cbase + tt * 16 + i;  // cbase = chunk start + 4 grp
                    C[i] = full ? idx : (idx < nt ? idx : KMX_BIG);
                }
                kmx_v4i acc[4];
#pragma unroll
                for (int c = 0; c < 4; c++)
#pragma unroll
                    for (int qt = 0; qt < 4; qt++)
                        acc[qt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[cur][c], B[qt][c], c == 0 ? C : acc[qt], 0, 0, 0);
#pragma unroll
                for (int qt = 0; qt < 4; qt++)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        k1[qt] = med3_i32(k0[qt], k1[qt], acc[qt][i]);
                        k0[qt] = min(k0[qt], acc[qt][i]);
                    }
            }
        };
        for (int ch = 0; ch < nch; ch++) {
            const int buf = ch & 1;
            if (ch + 1 < nch) fetch(ch + 1);
            if (live) {
                const int cbase = ch * KMX_T + 4 * grp;
                if ((ch + 1) * KMX_T <= nt) chunk(s_tr[buf], cbase, std::true_type{});
                else chunk(s_tr[buf], cbase, std::false_type{});
            }
            if (ch + 1 < nch) stage(buf ^ 1);
            __syncthreads();
        }
        if (!live) continue;
        // ---- merge the 4 lane groups holding each query, then lane l writes query qbase + l
#pragma unroll
        for (int m = 16; m <= 32; m <<= 1)
#pragma unroll
            for (int qt = 0; qt < 4; qt++) {
                const int p0 = __shfl_xor(k0[qt], m), p1 = __shfl_xor(k1[qt], m);
                const int n1 = min(max(k0[qt], p0), min(k1[qt], p1));
                k0[qt] = min(k0[qt], p0);
                k1[qt] = n1;
            }
        int a0 = k0[0], a1 = k1[0];
#pragma unroll
        for (int qt = 1; qt < 4; qt++)
            if (grp == qt) a0 = k0[qt], a1 = k1[qt];
        const int qpos = qbase + lane;
        if (qpos < nq) {
            const int qi = qlist ? qlist[(size_t)p * ql_stride + qpos] : qpos;
            const bool e0 = a0 > (1 << 21), e1 = a1 > (1 << 21);  // no train in the slot
            const int u0 = a0 + (1 << 20), u1 = a1 + (1 << 20);
            const size_t o = (size_t)p * out_stride + qi;
            out_idx[o] = make_int2(e0 ? -1 : (u0 & 8191), e1 ? -1 : (u1 & 8191));
            out_dist[o] = make_int2(e0 ? 0x7FFFFFFF : (u0 >> 13), e1 ? 0x7FFFFFFF : (u1 >> 13));
        }
    }
}
#endif  // ODO_TUNING

// ------------------------------------------------------------ FP4 form
// The same sign-vector product on v_mfma_scale_f32_16x16x128_f8f6f4 with e2m1
// operands: +1.0 (nibble 0x2) for a 0 bit, -1.0 (0xA) for a 1 bit, the query
// signs negated, unit scales. A 256-bit comparison is two k-steps of 128; the
// f32 sum is 2H - 256, exact, and the accumulator starts at 256 + idx / 8192, so
// the result is the key 2H + idx / 8192 (22 significant bits, exact in f32, every
// partial sum too), ordered as (H, idx). The keys are non-negative, so their bit
// patterns order as unsigned integers: top-2 is v_min_u32 + v_med3_u32 on the
// raw accumulator (no NaN canonicalisation), and the accumulator start is an
// integer add (the bits of 256 + idx / 8192 are 0x43800000 + 4 idx). Half the MFMAs of the
// int8 form, and a cheap expansion: the sign bit of nibble m of output dword j
// is descriptor bit j + 4m of the 32-bit word, so one word becomes its four
// dwords with one and + one shift-or each (A and B use the same permutation of
// the 256 bits, which leaves the dot product unchanged).
#define KF_T 128         // trains per LDS chunk (128 B per expanded train)
#define KF_PAD 0x45800000u    // 4096.0f: accumulator start of a train slot past the end
#define KF_EMPTY 0x46000000u  // 8192.0f
#define KF_BASE 0x43800000u   // 256.0f
#define KF_NONE 0x44800000u   // 1024.0f: keys at or above are no train
typedef float kf_v4f __attribute__((ext_vector_type(4)));
typedef int kf_v8i __attribute__((ext_vector_type(8)));

// one 32-bit descriptor word -> 32 e2m1 signs in 4 dwords
ODO_INLINE kmx_v4i kf_expand32(uint32_t w) {
    kmx_v4i r;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint32_t b;
        asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(b) : "v"(w & (0x11111111u << j)), "i"(3 - j), "s"(0x22222222u));
        r[j] = (int)b;
    }
    return r;
}
ODO_INLINE kf_v8i kf_op(kmx_v4i v) {
    kf_v8i r;
    r[0] = v[0], r[1] = v[1], r[2] = v[2], r[3] = v[3];
    r[4] = r[5] = r[6] = r[7] = 0;
    return r;
}

__global__ void __launch_bounds__(256, 3) k_knn2_f4(const uint8_t* __restrict__ qdesc, const int* __restrict__ qn,
                                                    size_t q_stride, const uint8_t* __restrict__ tdesc,
                                                    const int* __restrict__ tn, size_t t_stride,
                                                    int2* __restrict__ out_idx, int2* __restrict__ out_dist,
                                                    size_t out_stride, const int32_t* __restrict__ qlist,
                                                    const int* __restrict__ qcnt, size_t ql_stride, int npairs) {
    __builtin_amdgcn_s_setprio(ODO_KNN_PRIO);
    __shared__ __attribute__((aligned(16))) uint8_t s_tr[2][KF_T * 128];
    __shared__ int s_pre[KNN_MAXP + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, col = lane & 15;
    for (int i = tid; i < npairs; i += 256) {
        const int nq = qlist ? qcnt[i] : qn[i];
        s_pre[i + 1] = (nq + KMX_Q - 1) / KMX_Q;
    }
    if (tid == 0) s_pre[0] = 0;
    __syncthreads();
    if (tid == 0)
        for (int i = 1; i <= npairs; i++) s_pre[i] += s_pre[i - 1];
    __syncthreads();
    const int nact = s_pre[npairs];
    // staging role of this thread: train st_t of a chunk, words 4 st_h .. 4 st_h + 3
    const int st_t = tid >> 1, st_h = tid & 1;
    // XCD-aware item order: workgroups are dispatched round robin over the 8
    // XCDs (blockIdx % 8), so XCD x takes the contiguous item range
    // [x nact / 8, (x + 1) nact / 8) and strides its own workgroups over it. A
    // pair's query blocks (consecutive items) then stream the pair's train
    // descriptors through one XCD's L2 instead of up to five.
    int g_lo = 0, g_hi = nact, g_first = blockIdx.x, g_step = gridDim.x;
    if (gridDim.x >= 8) {
        const int x = blockIdx.x & 7;
        g_lo = (int)((long)nact * x / 8);
        g_hi = (int)((long)nact * (x + 1) / 8);
        g_first = g_lo + (blockIdx.x >> 3);
        g_step = (gridDim.x - x + 7) >> 3;  // workgroups on XCD x
    }
    for (int g = g_first; g < g_hi; g += g_step) {
        int lo = 0, hi = npairs;  // last pair with s_pre[p] <= g
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_pre[mid] <= g) lo = mid; else hi = mid;
        }
        const int p = lo, qb = g - s_pre[p];
        const int nq = qlist ? qcnt[p] : qn[p];
        const int nt = tn[p];
        const uint8_t* Q = qdesc + (size_t)p * q_stride;
        const uint8_t* T = tdesc + (size_t)p * t_stride;
        const int qbase = qb * KMX_Q + wave * 64;
        // ---- B operand: this wave's 64 queries, negated signs
        kmx_v4i B[4][2];
#pragma unroll
        for (int qt = 0; qt < 4; qt++) {
            const int qpos = qbase + qt * 16 + col;
            uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
            if (qpos < nq) {
                const int qi = qlist ? qlist[(size_t)p * ql_stride + qpos] : qpos;
                a = reinterpret_cast<const uint4*>(Q + (size_t)qi * 32)[0];
                b = reinterpret_cast<const uint4*>(Q + (size_t)qi * 32)[1];
            }
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int c = 0; c < 2; c++) {
                uint32_t h = 0;  // word 4 c + grp of k-step c, lane group grp
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if (k == 4 * c + grp) h = w[k];
                B[qt][c] = kf_expand32(~h);
            }
        }
        uint32_t k0[4], k1[4];
#pragma unroll
        for (int qt = 0; qt < 4; qt++) k0[qt] = k1[qt] = KF_EMPTY;
        const int nch = (nt + KF_T - 1) / KF_T;
        uint4 pf = make_uint4(0, 0, 0, 0);
        auto fetch = [&](int ch) {
            const int t = ch * KF_T + st_t;
            pf = t < nt ? *reinterpret_cast<const uint4*>(T + (size_t)t * 32 + 16 * st_h) : make_uint4(0, 0, 0, 0);
        };
        auto stage = [&](int buf) {
            uint8_t* dst = s_tr[buf] + st_t * 128;
            const uint32_t w[4] = {pf.x, pf.y, pf.z, pf.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int u = 4 * st_h + k;
                *reinterpret_cast<kmx_v4i*>(dst + ((u ^ (st_t & 7)) << 4)) = kf_expand32(w[k]);
            }
        };
        __syncthreads();  // the previous item's last chunk is no longer read
        if (nch > 0) {
            fetch(0);
            stage(0);
        }
        __syncthreads();
        const bool live = qbase < nq;  // wave-uniform: this wave holds queries
        // one chunk of 128 trains: 8 tiles of 16 trains x 2 k-steps x 4 query tiles
        auto chunk = [&](const uint8_t* src, int cbase, auto full_tag) {
            constexpr bool full = decltype(full_tag)::value;
            kmx_v4i A[2][2];
#pragma unroll
            for (int c = 0; c < 2; c++)
                A[0][c] = *reinterpret_cast<const kmx_v4i*>(src + col * 128 + (((4 * c + grp) ^ (col & 7)) << 4));
#pragma unroll
            for (int tt = 0; tt < KF_T / 16; tt++) {
                const int cur = tt & 1;
                if (tt + 1 < KF_T / 16) {
                    const int r = (tt + 1) * 16 + col;  // train row of this lane's next A operand
#pragma unroll
                    for (int c = 0; c < 2; c++)
                        A[cur ^ 1][c] = *reinterpret_cast<const kmx_v4i*>(src + r * 128 + (((4 * c + grp) ^ (col & 7)) << 4));
                }
                kmx_v4i Cb;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int idx = cbase + tt * 16 + i;  // cbase = chunk start + 4 grp
                    Cb[i] = (full || idx < nt) ? (int)(KF_BASE + 4u * (uint32_t)idx) : (int)KF_PAD;
                }
                const kf_v4f C = __builtin_bit_cast(kf_v4f, Cb);
                kf_v4f acc[4];
#pragma unroll
                for (int c = 0; c < 2; c++)
#pragma unroll
                    for (int qt = 0; qt < 4; qt++)
                        acc[qt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                            kf_op(A[cur][c]), kf_op(B[qt][c]), c == 0 ? C : acc[qt], 4, 4, 0, 127, 0, 127);
                // top-2 over two new keys at a time (k0 <= k1 holds throughout):
                // the second smallest of {k0, k1, x0, x1} is min(k1, med3(k0, x0, x1))
                // and the smallest min3(k0, x0, x1): 3 ops per 2 keys instead of 4
#pragma unroll
                for (int qt = 0; qt < 4; qt++)
#pragma unroll
                    for (int i = 0; i < 4; i += 2) {
                        const uint32_t x0 = __float_as_uint(acc[qt][i]), x1 = __float_as_uint(acc[qt][i + 1]);
                        const uint32_t m = max(min(k0[qt], x0), min(max(k0[qt], x0), x1));  // v_med3_u32
                        k1[qt] = min(k1[qt], m);
                        // v_min3_u32 as inline asm (the optimiser would share
                        // min(k0, x0) with the med3 and issue two v_min_u32). m is
                        // a dependency only: the asm follows the med3, which
                        // already read x0 / x1 past the MFMA's result hazard.
                        uint32_t n0;
                        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(n0) : "v"(k0[qt]), "v"(x0), "v"(x1), "v"(m));
                        k0[qt] = n0;
                    }
            }
        };
        for (int ch = 0; ch < nch; ch++) {
            const int buf = ch & 1;
            if (ch + 1 < nch) fetch(ch + 1);
            if (live) {
                const int cbase = ch * KF_T + 4 * grp;
                if ((ch + 1) * KF_T <= nt) chunk(s_tr[buf], cbase, std::true_type{});
                else chunk(s_tr[buf], cbase, std::false_type{});
            }
            if (ch + 1 < nch) stage(buf ^ 1);
            __syncthreads();
        }
        if (!live) continue;
        // ---- merge the 4 lane groups holding each query, then lane l writes query qbase + l
#pragma unroll
        for (int m = 16; m <= 32; m <<= 1)
#pragma unroll
            for (int qt = 0; qt < 4; qt++) {
                const uint32_t p0 = __shfl_xor(k0[qt], m), p1 = __shfl_xor(k1[qt], m);
                const uint32_t n1 = min(max(k0[qt], p0), min(k1[qt], p1));
                k0[qt] = min(k0[qt], p0);
                k1[qt] = n1;
            }
        uint32_t a0 = k0[0], a1 = k1[0];
#pragma unroll
        for (int qt = 1; qt < 4; qt++)
            if (grp == qt) a0 = k0[qt], a1 = k1[qt];
        const int qpos = qbase + lane;
        if (qpos < nq) {
            const int qi = qlist ? qlist[(size_t)p * ql_stride + qpos] : qpos;
            // no train in the slot: a pad row's key is 4096 + (2H - 256), real keys are < 513
            const bool e0 = a0 >= KF_NONE, e1 = a1 >= KF_NONE;
            const int u0 = (int)(__uint_as_float(a0) * 8192.0f), u1 = (int)(__uint_as_float(a1) * 8192.0f);  // 16384 H + idx
            const size_t o = (size_t)p * out_stride + qi;
            out_idx[o] = make_int2(e0 ? -1 : (u0 & 8191), e1 ? -1 : (u1 & 8191));
            out_dist[o] = make_int2(e0 ? 0x7FFFFFFF : (u0 >> 14), e1 ? 0x7FFFFFFF : (u1 >> 14));
        }
    }
}

// ============================================================ libstdc++ std::sort emulation
// Exactly the GNU introsort (std::__introsort_loop + __final_insertion_sort,
// threshold 16, median-of-3 pivot, unguarded Hoare partition, heap fallback) on
// 64-bit (key = distance bits, payload = position) elements compared by key
// only: reproduces the unstable order of std::sort(vector<DMatch>) in
// ransac.cpp:199 (App. B.4). Runs on one lane over an LDS/global array.
struct SortEl {
    uint32_t key;  // float bits of a non-negative distance (monotonic)
    uint32_t val;
};

template <typename A>
ODO_INLINE void st_swap(A a, int i, int j) {
    SortEl t = a[i];
    a[i] = a[j];
    a[j] = t;
}

template <typename A>
ODO_INLINE void st_move_median_to_first(A a, int result, int x, int y, int z) {
    const uint32_t ax = a[x].key, ay = a[y].key, az = a[z].key;
    if (ax < ay) {
        if (ay < az) st_swap(a, result, y);
        else if (ax < az) st_swap(a, result, z);
        else st_swap(a, result, x);
    } else if (ax < az) st_swap(a, result, x);
    else if (ay < az) st_swap(a, result, z);
    else st_swap(a, result, y);
}

template <typename A>
ODO_INLINE int st_unguarded_partition(A a, int first, int last, int pivot) {
    const uint32_t pk = a[pivot].key;
    while (true) {
        while (a[first].key < pk) ++first;
        --last;
        while (pk < a[last].key) --last;
        if (!(first < last)) return first;
        st_swap(a, first, last);
        ++first;
    }
}

template <typename A>
ODO_INLINE void st_adjust_heap(A a, int first, int holeIndex, int len, SortEl value) {
    const int topIndex = holeIndex;
    int secondChild = holeIndex;
    while (secondChild < (len - 1) / 2) {
        secondChild = 2 * (secondChild + 1);
        if (a[first + secondChild].key < a[first + secondChild - 1].key) secondChild--;
        a[first + holeIndex] = a[first + secondChild];
        holeIndex = secondChild;
    }
    if ((len & 1) == 0 && secondChild == (len - 2) / 2) {
        secondChild = 2 * (secondChild + 1);
        a[first + holeIndex] = a[first + secondChild - 1];
        holeIndex = secondChild - 1;
    }
    // __push_heap
    int parent = (holeIndex - 1) / 2;
    while (holeIndex > topIndex && a[first + parent].key < value.key) {
        a[first + holeIndex] = a[first + parent];
        holeIndex = parent;
        parent = (holeIndex - 1) / 2;
    }
    a[first + holeIndex] = value;
}

template <typename A>
ODO_INLINE void st_heap_sort_range(A a, int first, int middle, int last) {
    // std::__partial_sort(first, middle=last, last): __heap_select + __sort_heap
    const int len = middle - first;
    if (len >= 2) {
        for (int parent = (len - 2) / 2;; parent--) {
            SortEl v = a[first + parent];
            st_adjust_heap(a, first, parent, len, v);
            if (parent == 0) break;
        }
    }
    for (int i = middle; i < last; ++i)
        if (a[i].key < a[first].key) {
            SortEl v = a[i];
            a[i] = a[first];
            st_adjust_heap(a, first, 0, len, v);
        }
    for (int l2 = middle; l2 - first > 1;) {
        --l2;
        SortEl v = a[l2];
        a[l2] = a[first];
        st_adjust_heap(a, first, 0, l2 - first, v);
    }
}

template <typename A>
ODO_INLINE void st_insertion_sort(A a, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        SortEl val = a[i];
        if (val.key < a[first].key) {
            for (int k = i; k > first; --k) a[k] = a[k - 1];
            a[first] = val;
        } else {
            int next = i - 1, cur = i;
            while (val.key < a[next].key) {
                a[cur] = a[next];
                cur = next;
                --next;
            }
            a[cur] = val;
        }
    }
}

template <typename A>
ODO_INLINE void st_unguarded_insertion_sort(A a, int first, int last) {
    for (int i = first; i != last; ++i) {
        SortEl val = a[i];
        int next = i - 1, cur = i;
        while (val.key < a[next].key) {
            a[cur] = a[next];
            cur = next;
            --next;
        }
        a[cur] = val;
    }
}

template <typename A>
ODO_INLINE void gnu_sort(A a, int n) {
    if (n < 2) return;
    // __introsort_loop with an explicit stack (recursion on the right part)
    int lg = 31 - __builtin_clz((unsigned)n);
    int stk_first[64], stk_last[64], stk_depth[64];
    int sp = 0;
    stk_first[sp] = 0;
    stk_last[sp] = n;
    stk_depth[sp] = 2 * lg;
    sp++;
    while (sp > 0) {
        sp--;
        int first = stk_first[sp], last = stk_last[sp], depth = stk_depth[sp];
        while (last - first > 16) {
            if (depth == 0) {
                st_heap_sort_range(a, first, last, last);
                break;
            }
            --depth;
            const int mid = first + (last - first) / 2;
            st_move_median_to_first(a, first, first + 1, mid, last - 1);
            const int cut = st_unguarded_partition(a, first + 1, last, first);
            // recurse on [cut, last) first (it is processed before the left loop
            // continues in libstdc++, but the two ranges are disjoint, so order
            // of processing does not change the result)
            stk_first[sp] = cut;
            stk_last[sp] = last;
            stk_depth[sp] = depth;
            sp++;
            last = cut;
        }
    }
    if (n > 16) {
        st_insertion_sort(a, 0, 16);
        st_unguarded_insertion_sort(a, 16, n);
    } else st_insertion_sort(a, 0, n);
}

// ---- workgroup-parallel std::sort (identical permutation to gnu_sort) -------
// Level-synchronous introsort: every range of a level is partitioned at once.
// A Hoare partition (pivot key pk at `first`) swaps the k-th element from the
// left with key >= pk against the k-th from the right with key <= pk for all
// k < k*, k* = the first k where those stops cross, and cuts at the k*-th left
// stop; ranks come from prefix counts over the level. Ranges are disjoint, so
// the order libstdc++ recurses in does not matter. __final_insertion_sort never
// moves an element across a cut (keys left of a cut are <= keys right of it),
// so it equals a stable sort inside every final range, done one range per
// thread.
#define PS_MAXR 512

struct PSortRanges {
    int f[PS_MAXR], l[PS_MAXR], d[PS_MAXR], pk[PS_MAXR], ks[PS_MAXR];
    int gs[PS_MAXR], ge[PS_MAXR], ls[PS_MAXR], le[PS_MAXR], cut[PS_MAXR];
    int nf[2 * PS_MAXR], nd[2 * PS_MAXR];
    int nr;
    int ws[16][2];
};

static inline size_t psort_lds_bytes(int pw) {
    return (size_t)pw * (8 + 2 + 2 + 2 + 1) + sizeof(PSortRanges) + 64;
}

// exclusive block scan of two per-thread counts
ODO_INLINE int2 block_scan2(int a, int b, int (*ws)[2]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int ia = a, ib = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(ia, o), y = __shfl_up(ib, o);
        if (lane >= o) {
            ia += x;
            ib += y;
        }
    }
    if (lane == 63) {
        ws[w][0] = ia;
        ws[w][1] = ib;
    }
    __syncthreads();
    int ba = 0, bb = 0;
    for (int k = 0; k < w; k++) {
        ba += ws[k][0];
        bb += ws[k][1];
    }
    __syncthreads();
    return make_int2(ba + ia - a, bb + ib - b);
}

// range of position j (j in [f+1, l) of an active range), or -1
ODO_INLINE int psort_find(const PSortRanges& R, int nr, int j) {
    int lo = 0, hi = nr - 1, r = -1;
    while (lo <= hi) {
        const int m = (lo + hi) >> 1;
        if (R.f[m] < j) {
            r = m;
            lo = m + 1;
        } else hi = m - 1;
    }
    if (r < 0 || j >= R.l[r] || R.d[r] < 0) return -1;
    return r;
}

ODO_INLINE void block_gnu_sort(SortEl* A, int n, uint8_t* work, PSortRanges& R) {
    const int t = threadIdx.x, T = blockDim.x;
    if (n < 2) return;
    uint16_t* rid = reinterpret_cast<uint16_t*>(work);
    uint16_t* posL = rid + n;
    uint16_t* posR = posL + n;
    uint8_t* cutf = reinterpret_cast<uint8_t*>(posR + n);  // range boundaries
    for (int j = t; j < n; j += T) cutf[j] = j == 0;
    if (t == 0) {
        R.nr = 0;
        if (n > 16) {
            R.f[0] = 0;
            R.l[0] = n;
            R.d[0] = 2 * (31 - __builtin_clz((unsigned)n));
            R.nr = 1;
        }
    }
    __syncthreads();
    const int c = (n + T - 1) / T;
    const int j0 = min(n, t * c), j1 = min(n, j0 + c);
    while (R.nr > 0) {
        const int nr = R.nr;
        // pivot: median of three moved to `first`; depth 0 -> heap sort (range done)
        for (int r = t; r < nr; r += T) {
            const int f = R.f[r], l = R.l[r], d = R.d[r];
            if (d == 0) {
                st_heap_sort_range(A, f, l, l);
                R.d[r] = -1;
            } else {
                R.d[r] = d - 1;
                st_move_median_to_first(A, f, f + 1, f + (l - f) / 2, l - 1);
                R.pk[r] = (int)A[f].key;
                R.ks[r] = 0;
            }
        }
        __syncthreads();
        for (int j = t; j < n; j += T) {
            const int r = psort_find(R, nr, j);
            rid[j] = r < 0 ? 0xffff : (uint16_t)r;
        }
        __syncthreads();
        // left stops: key >= pk, right stops: key <= pk (over [f+1, l))
        int cg = 0, cl = 0;
        for (int j = j0; j < j1; j++) {
            const int r = rid[j];
            if (r == 0xffff) continue;
            const uint32_t k = A[j].key, pk = (uint32_t)R.pk[r];
            cg += k >= pk;
            cl += k <= pk;
        }
        const int2 base = block_scan2(cg, cl, R.ws);
        int rg = base.x, rl = base.y;
        for (int j = j0; j < j1; j++) {
            const int r = rid[j];
            if (r == 0xffff) continue;
            if (j == R.f[r] + 1) {
                R.gs[r] = rg;
                R.ls[r] = rl;
            }
            const uint32_t k = A[j].key, pk = (uint32_t)R.pk[r];
            rg += k >= pk;
            rl += k <= pk;
            if (j == R.l[r] - 1) {
                R.ge[r] = rg;
                R.le[r] = rl;
            }
        }
        __syncthreads();
        rg = base.x;
        rl = base.y;
        for (int j = j0; j < j1; j++) {
            const int r = rid[j];
            if (r == 0xffff) continue;
            const uint32_t k = A[j].key, pk = (uint32_t)R.pk[r];
            const int f = R.f[r];
            if (k >= pk) posL[f + (rg - R.gs[r])] = (uint16_t)j;
            rg += k >= pk;
            rl += k <= pk;
            if (k <= pk) posR[f + (R.le[r] - rl)] = (uint16_t)j;
        }
        __syncthreads();
        // k* = #{k : posL[k] < posR[k]} (monotone in k)
        for (int q = t; q + 1 < n; q += T) {
            const int r = rid[q + 1];
            if (r == 0xffff) continue;
            const int k = q - R.f[r];
            const int m = min(R.ge[r] - R.gs[r], R.le[r] - R.ls[r]);
            if (k < m && posL[q] < posR[q]) atomicAdd(&R.ks[r], 1);
        }
        __syncthreads();
        for (int q = t; q + 1 < n; q += T) {
            const int r = rid[q + 1];
            if (r == 0xffff) continue;
            const int k = q - R.f[r];
            if (k < R.ks[r]) {
                const int a = posL[q], b = posR[q];
                const SortEl x = A[a];
                A[a] = A[b];
                A[b] = x;
            }
        }
        for (int r = t; r < nr; r += T) {
            int f = -1, cut = -1, l = -1;
            if (R.d[r] >= 0) {
                // the left scan stops at the k*-th original left stop, or
                // earlier at R[k*-1], which now holds a swapped-in key >= pk
                f = R.f[r];
                l = R.l[r];
                const int ks = R.ks[r];
                cut = l;
                if (ks < R.ge[r] - R.gs[r]) cut = posL[f + ks];
                if (ks > 0) cut = min(cut, (int)posR[f + ks - 1]);
                cutf[cut] = 1;
            }
            // children with more than 16 elements continue at the next level
            R.nf[2 * r] = (cut >= 0 && cut - f > 16) ? f : -1;
            R.nf[2 * r + 1] = (cut >= 0 && l - cut > 16) ? cut : -1;
            R.cut[r] = cut;
        }
        __syncthreads();
        // compact the next level's ranges (in position order)
        const int m2 = 2 * nr;
        const int cc = (m2 + T - 1) / T;
        const int q0 = min(m2, t * cc), q1 = min(m2, q0 + cc);
        int cnt = 0;
        for (int q = q0; q < q1; q++) cnt += R.nf[q] >= 0;
        const int2 nb = block_scan2(cnt, 0, R.ws);
        int o = nb.x;
        int nf_[8], nl_[8], nd_[8], nq = 0;
        for (int q = q0; q < q1; q++) {
            if (R.nf[q] < 0) continue;
            const int r = q >> 1;
            nf_[nq & 7] = (q & 1) ? R.cut[r] : R.f[r];
            nl_[nq & 7] = (q & 1) ? R.l[r] : R.cut[r];
            nd_[nq & 7] = R.d[r];
            nq++;
        }
        __syncthreads();
        for (int i = 0; i < nq && i < 8; i++) {
            R.f[o + i] = nf_[i];
            R.l[o + i] = nl_[i];
            R.d[o + i] = nd_[i];
        }
        if (t == T - 1) R.nr = o + nq;
        __syncthreads();
    }
    // __final_insertion_sort == stable sort inside each final range
    for (int j = t; j < n; j += T) {
        if (!cutf[j]) continue;
        int e = j + 1;
        while (e < n && !cutf[e]) e++;
        for (int i = j + 1; i < e; i++) {
            const SortEl v = A[i];
            int k = i;
            while (k > j && v.key < A[k - 1].key) {
                A[k] = A[k - 1];
                k--;
            }
            A[k] = v;
        }
    }
    __syncthreads();
}

#define PM_THREADS 256

// ============================================================ VO landmarks
// Tracking::UpdateLastFrame's visual-odometry landmarks of every query frame
// (F1 of pair p, tracking.cpp:146-190): the K smallest (z, index) pairs among
// z > 0, K = min(valid, max(#(z <= th) + 1, 101)): with #(z <= th) >= 100 the
// points within th plus the nearest one beyond, else a bitonic sort in LDS.
// Outputs the landmark bit set and the landmark keypoints in index order.
// Matcher::KnnMatch drops every query without a landmark (matcher.cpp:70-72),
// so kNN-2 runs on this list alone; its matches are unchanged.
__global__ void __launch_bounds__(PM_THREADS) k_vo_lm(const float* __restrict__ xyz, const int* __restrict__ nkp,
                                                      int kp_cap, int slot0, float th_depth_m,
                                                      uint32_t* __restrict__ lm_g, int lm_words,
                                                      int32_t* __restrict__ qlist, int* __restrict__ qcnt) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];  // pw entries
    __shared__ int s_total_valid, s_cle, s_w[PM_THREADS / 64];
    __shared__ unsigned long long s_min;
    __shared__ uint32_t bits[(8192 + 31) / 32];
    const int p = blockIdx.x, t = threadIdx.x;
    const int s1 = slot0 + p;
    const int n1 = nkp[s1];
    const float* X1 = xyz + (size_t)s1 * kp_cap * 3;
    int cv = 0, cle = 0;
    for (int i = t; i < n1; i += PM_THREADS) {
        const float z = X1[3 * i + 2];
        if (z > 0) {
            cv++;
            cle += z <= th_depth_m;
        }
    }
    if (t == 0) {
        s_total_valid = 0;
        s_cle = 0;
    }
    for (int i = t; i < lm_words; i += PM_THREADS) bits[i] = 0;
    __syncthreads();
    atomicAdd(&s_total_valid, cv);
    atomicAdd(&s_cle, cle);
    __syncthreads();
    const int valid = s_total_valid;
    int K = s_cle + 1 > 101 ? s_cle + 1 : 101;
    if (K > valid) K = valid;
    if (s_cle >= 100) {
        // the common case, K = #(z <= th) + 1 (or all valid): every point with
        // z <= th plus the smallest (z, index) beyond th — no sort needed
        if (t == 0) s_min = ~0ull;
        __syncthreads();
        uint64_t mk = ~0ull;
        for (int i = t; i < n1; i += PM_THREADS) {
            const float z = X1[3 * i + 2];
            if (z > 0) {
                if (z <= th_depth_m)
                    atomicOr(&bits[i >> 5], 1u << (i & 31));
                else {
                    const uint64_t key = ((uint64_t)__float_as_uint(z) << 32) | (uint32_t)i;
                    mk = key < mk ? key : mk;
                }
            }
        }
        atomicMin(&s_min, mk);
        __syncthreads();
        if (t == 0 && K > s_cle && s_min != ~0ull) {
            const int i = (int)(uint32_t)s_min;
            bits[i >> 5] |= 1u << (i & 31);
        }
        __syncthreads();
    } else {
    // rank selection: sort (z_bits << 32 | i) ascending (z > 0: the float bits order as integers)
    int pw = 1;
    while (pw < n1) pw <<= 1;
    for (int i = t; i < pw; i += PM_THREADS) {
        uint64_t key = ~0ull;
        if (i < n1) {
            const float z = X1[3 * i + 2];
            if (z > 0) key = ((uint64_t)__float_as_uint(z) << 32) | (uint32_t)i;
        }
        sk[i] = key;
    }
    __syncthreads();
    for (int kk = 2; kk <= pw; kk <<= 1)
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            for (int i = t; i < pw; i += PM_THREADS) {
                const int ixj = i ^ jj;
                if (ixj > i) {
                    const uint64_t a = sk[i], b = sk[ixj];
                    const bool up = (i & kk) == 0;
                    if ((a > b) == up) {
                        sk[i] = b;
                        sk[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    for (int r = t; r < K; r += PM_THREADS) {
        const int i = (int)(uint32_t)sk[r];
        atomicOr(&bits[i >> 5], 1u << (i & 31));
    }
    __syncthreads();
    }
    for (int i = t; i < lm_words; i += PM_THREADS) lm_g[(size_t)p * lm_words + i] = bits[i];
    // the landmark keypoints in index order
    const int wave = t >> 6, lane = t & 63;
    int base = 0;
    for (int c0 = 0; c0 < n1; c0 += PM_THREADS) {
        const int i = c0 + t;
        const bool keep = i < n1 && ((bits[i >> 5] >> (i & 31)) & 1u);
        const uint64_t bal = __ballot(keep);
        if (lane == 0) s_w[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < PM_THREADS / 64; w++) {
            if (w < wave) before += s_w[w];
            tot += s_w[w];
        }
        if (keep)
            qlist[(size_t)p * kp_cap + base + before +
                  __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0))] = i;
        base += tot;
        __syncthreads();
    }
    if (t == 0) qcnt[p] = base;
}

// ============================================================ per-pair match stage
// One workgroup (256 threads) per pair (F1 = previous frame, F2 = current).
// Outputs: good matches sorted per std::sort (query/train/distance), counts,
// f2_src[i2] = F1 index whose landmark sits in F2 slot i2 (-1 if none).
__global__ void __launch_bounds__(PM_THREADS) k_pair_match(
    const int2* __restrict__ knn_idx, const int2* __restrict__ knn_dist, size_t knn_stride,
    const float* __restrict__ xyz, const int* __restrict__ nkp, int kp_cap, int slot0, float ratio,
    const uint32_t* __restrict__ lm_g, int lm_words, int nsplit, size_t split_stride, int check_depth,
    odo_dmatch* __restrict__ matches,
    int* __restrict__ n_matches,
    SortEl* __restrict__ good, int* __restrict__ n_good, int32_t* __restrict__ f2_src,
    uint64_t* __restrict__ sort_scratch, int match_cap) {
    __builtin_amdgcn_s_setprio(ODO_WAVE_PRIO);  // latency-bound: issue ahead of co-resident extraction waves
    __shared__ int s_cnt[PM_THREADS];
    extern __shared__ __attribute__((aligned(16))) uint64_t dyn_lds[];  // pw entries
    const int p = blockIdx.x;                  // pair index
    const int s1 = slot0 + p, s2 = slot0 + p + 1;
    const int n1 = nkp[s1], n2 = nkp[s2];
    const int t = threadIdx.x;
    const float* X1 = xyz + (size_t)s1 * kp_cap * 3;
    const float* X2 = xyz + (size_t)s2 * kp_cap * 3;
    (void)sort_scratch;
    int32_t* src = f2_src + (size_t)p * kp_cap;
    for (int i = t; i < n2; i += PM_THREADS) src[i] = -1;
    // ---- VO landmarks on F1 (UpdateLastFrame, tracking.cpp:146-190): the bit
    // set k_vo_lm computed before kNN-2 (queries without one have no kNN-2 output)
    int pw = 1;
    while (pw < n1) pw <<= 1;
    __shared__ uint32_t lm_bits[(8192 + 31) / 32];
    for (int i = t; i < lm_words; i += PM_THREADS) lm_bits[i] = lm_g[(size_t)p * lm_words + i];
    __syncthreads();
    // ---- ratio test + bookkeeping in query order (all F1 landmarks are fresh
    // VO landmarks with 0 observations and F2 starts empty, so no match is
    // skipped by the Observations()>0 rule; the last query wins a train slot).
    const int2* KI = knn_idx + (size_t)p * knn_stride;
    const int2* KD = knn_dist + (size_t)p * knn_stride;
    odo_dmatch* M = matches + (size_t)p * match_cap;
    int base = 0;
    for (int c0 = 0; c0 < n1; c0 += PM_THREADS) {
        const int i = c0 + t;
        bool acc = false;
        int2 I = make_int2(-1, -1), D = make_int2(0, 0);
        if (i < n1 && ((lm_bits[i >> 5] >> (i & 31)) & 1)) {  // kNN-2 ran on landmark queries only
            // the train splits' top-2 lists merged: the two smallest (distance, index) keys
            uint32_t k0 = 0xFFFFFFFFu, k1 = 0xFFFFFFFFu;
            for (int h = 0; h < nsplit; h++) {
                const int2 Ih = KI[(size_t)h * split_stride + i], Dh = KD[(size_t)h * split_stride + i];
                const uint32_t a = Ih.x >= 0 ? ((uint32_t)Dh.x << 20) | (uint32_t)Ih.x : 0xFFFFFFFFu;
                const uint32_t b = Ih.y >= 0 ? ((uint32_t)Dh.y << 20) | (uint32_t)Ih.y : 0xFFFFFFFFu;
                // two sorted pairs: second smallest = min(max(k0, a), k1, b)
                k1 = min(max(k0, a), min(k1, b));
                k0 = min(k0, a);
            }
            I = make_int2(k0 == 0xFFFFFFFFu ? -1 : (int)(k0 & 0xFFFFF), k1 == 0xFFFFFFFFu ? -1 : (int)(k1 & 0xFFFFF));
            D = make_int2(k0 == 0xFFFFFFFFu ? 0x7FFFFFFF : (int)(k0 >> 20), k1 == 0xFFFFFFFFu ? 0x7FFFFFFF : (int)(k1 >> 20));
            if (I.x >= 0) {
                const float d0 = (float)D.x, d1 = (float)D.y;
                acc = d0 < ratio * d1;
            }
        }
        s_cnt[t] = acc;
        __syncthreads();
        for (int off = 1; off < PM_THREADS; off <<= 1) {
            int a = t >= off ? s_cnt[t - off] : 0;
            __syncthreads();
            s_cnt[t] += a;
            __syncthreads();
        }
        const int incl = s_cnt[t];
        const int tot = s_cnt[PM_THREADS - 1];
        if (acc) {
            const int pos = base + incl - 1;
            if (pos < match_cap) M[pos] = odo_dmatch{i, I.x, 0, (float)D.x};
            atomicMax(&src[I.x], i);
        }
        base += tot;
        __syncthreads();
    }
    const int nm = base < match_cap ? base : match_cap;
    if (t == 0) n_matches[p] = nm;
    __syncthreads();
    // ---- good-match filter (ransac.cpp:175-189), order preserved
    SortEl* G = good + (size_t)p * match_cap;
    int gbase = 0;
    for (int c0 = 0; c0 < nm; c0 += PM_THREADS) {
        const int i = c0 + t;
        bool g = false;
        odo_dmatch m;
        if (i < nm) {
            m = M[i];
            const float zs = X1[3 * m.queryIdx + 2], zt = X2[3 * m.trainIdx + 2];
            g = true;
            if (check_depth) {
                if (__builtin_isnan(zs) || __builtin_isnan(zt)) g = false;
                if (zs <= 0 || zt <= 0) g = false;
            }
        }
        s_cnt[t] = g;
        __syncthreads();
        for (int off = 1; off < PM_THREADS; off <<= 1) {
            int a = t >= off ? s_cnt[t - off] : 0;
            __syncthreads();
            s_cnt[t] += a;
            __syncthreads();
        }
        const int incl = s_cnt[t];
        const int tot = s_cnt[PM_THREADS - 1];
        if (g) G[gbase + incl - 1] = SortEl{__float_as_uint(m.distance), (uint32_t)i};
        gbase += tot;
        __syncthreads();
    }
    // ---- std::sort(vGoodMatches) by distance (ransac.cpp:199): exact
    // libstdc++ permutation, workgroup-parallel, in LDS
    SortEl* Gl = reinterpret_cast<SortEl*>(dyn_lds);
    for (int i = t; i < gbase; i += PM_THREADS) Gl[i] = G[i];
    if (t == 0) n_good[p] = gbase;
    __syncthreads();
    block_gnu_sort(Gl, gbase, reinterpret_cast<uint8_t*>(dyn_lds) + (size_t)pw * 8,
                   *reinterpret_cast<PSortRanges*>(reinterpret_cast<uint8_t*>(dyn_lds) +
                                                  (((size_t)pw * 15 + 63) & ~(size_t)63)));
    for (int i = t; i < gbase; i += PM_THREADS) G[i] = Gl[i];
    (void)n2;
}

// Ransac::DepthCovariance latches on its first call in the process
// (ransac.cpp:416-421): z0 = source z of the first sorted good match whose
// target.x != 0 in the first pair that reaches ComputeInliersAndError.
__global__ void k_latch(double* __restrict__ latch, const SortEl* __restrict__ good, const int* __restrict__ n_good,
                        const int* __restrict__ n_matches, const odo_dmatch* __restrict__ matches,
                        const float* __restrict__ xyz, int kp_cap, int slot0, int npairs, int match_cap,
                        int min_inl, int sample_size, int iterations, const int* __restrict__ pair_valid,
                        int* __restrict__ set_flag) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    // set_flag (page-locked host memory, may be null): 1 once the latch holds
    // a value, so the host can stop ordering later batches' latch kernels
    if (!__builtin_isnan(*latch)) {
        if (set_flag) *set_flag = 1;
        return;
    }
    for (int p = 0; p < npairs; p++) {
        if (!pair_valid[p]) continue;
        if (n_matches[p] < 20 || n_matches[p] < min_inl) continue;
        const int ng = n_good[p];
        if (ng < min_inl) continue;
        (void)iterations;
        (void)sample_size;
        const SortEl* G = good + (size_t)p * match_cap;
        const odo_dmatch* M = matches + (size_t)p * match_cap;
        const float* X1 = xyz + (size_t)(slot0 + p) * kp_cap * 3;
        const float* X2 = xyz + (size_t)(slot0 + p + 1) * kp_cap * 3;
        for (int k = 0; k < ng; k++) {
            const odo_dmatch m = M[G[k].val];
            if (X1[3 * m.queryIdx + 2] == 0.0f || X2[3 * m.trainIdx] == 0.0f) continue;
            const double z = (double)X1[3 * m.queryIdx + 2];
            const double sd = 0.01 * z * z;
            *latch = sd * sd;
            if (set_flag) *set_flag = 1;
            return;
        }
    }
}

}  // namespace odo

namespace odo {
void launch_knn2(hipStream_t st, const uint8_t* q, const int* qn, size_t q_stride, const uint8_t* t, const int* tn,
                 size_t t_stride, int2* idx, int2* dist, size_t out_stride, int max_q, int npairs,
                 const int32_t* qlist, const int* qcnt, size_t ql_stride, int nsplit, size_t split_stride) {
    static int resident = 0;  // workgroups of one full round (occupancy x CUs)
    if (!resident) {
        int dev = 0, cus = 256, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_knn2, KNN_TH, 0);
        // ODO_KNN_WG_PER_CU < occupancy leaves wave slots to co-running kernels
        if (const char* e = odo_knob("ODO_KNN_WG_PER_CU")) per_cu = std::min(std::max(1, atoi(e)), std::max(1, per_cu));
        resident = std::max(1, per_cu) * cus;
    }
    const int qblocks = (max_q + KNN_Q - 1) / KNN_Q;
    const int nitems = qblocks * npairs * nsplit;
    if (nitems <= 0) return;
    if (npairs > KNN_MAXP) {  // the item prefix is per launch: split larger batches
        launch_knn2(st, q, qn, q_stride, t, tn, t_stride, idx, dist, out_stride, max_q, KNN_MAXP, qlist, qcnt,
                    ql_stride, nsplit, split_stride);
        launch_knn2(st, q + KNN_MAXP * q_stride, qn + KNN_MAXP, q_stride, t + KNN_MAXP * t_stride, tn + KNN_MAXP,
                    t_stride, idx + KNN_MAXP * out_stride, dist + KNN_MAXP * out_stride, out_stride, max_q,
                    npairs - KNN_MAXP, qlist ? qlist + KNN_MAXP * ql_stride : nullptr, qcnt ? qcnt + KNN_MAXP : nullptr,
                    ql_stride, nsplit, split_stride);
        return;
    }
    dim3 g(std::min(nitems, resident));
    hipLaunchKernelGGL(k_knn2, g, dim3(KNN_TH), 0, st, q, qn, q_stride, t, tn, t_stride, idx, dist, out_stride, qlist,
                       qcnt, ql_stride, split_stride, npairs, qblocks, nsplit);
}
void launch_knn2_mx(hipStream_t st, const uint8_t* q, const int* qn, size_t q_stride, const uint8_t* t, const int* tn,
                    size_t t_stride, int2* idx, int2* dist, size_t out_stride, int max_q, int npairs,
                    const int32_t* qlist, const int* qcnt, size_t ql_stride, int fmt) {
    const bool f4 = fmt == KNN_FMT_F4;
    static int resident[2] = {0, 0};  // workgroups of one full round (occupancy x CUs), per kernel
    if (!resident[f4]) {
        int dev = 0, cus = 256, per_cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#ifdef ODO_TUNING
        const void* kf = f4 ? (const void*)k_knn2_f4 : (const void*)k_knn2_mx;
#else
        const void* kf = (const void*)k_knn2_f4;
#endif
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, 256, 0);
        // ODO_KNN_WG_PER_CU (tuning) < occupancy leaves register room to the
        // co-running extraction kernels
        if (const char* e = odo_knob("ODO_KNN_WG_PER_CU")) per_cu = std::min(std::max(1, atoi(e)), std::max(1, per_cu));
        resident[f4] = std::max(1, per_cu) * cus;
    }
    if (npairs <= 0 || max_q <= 0) return;
    if (npairs > KNN_MAXP) {  // the item prefix is per launch: split larger batches
        launch_knn2_mx(st, q, qn, q_stride, t, tn, t_stride, idx, dist, out_stride, max_q, KNN_MAXP, qlist, qcnt,
                       ql_stride, fmt);
        launch_knn2_mx(st, q + KNN_MAXP * q_stride, qn + KNN_MAXP, q_stride, t + KNN_MAXP * t_stride, tn + KNN_MAXP,
                       t_stride, idx + KNN_MAXP * out_stride, dist + KNN_MAXP * out_stride, out_stride, max_q,
                       npairs - KNN_MAXP, qlist ? qlist + KNN_MAXP * ql_stride : nullptr,
                       qcnt ? qcnt + KNN_MAXP : nullptr, ql_stride, fmt);
        return;
    }
    const int items = npairs * ((max_q + KMX_Q - 1) / KMX_Q);  // upper bound; the kernel counts the real ones
    const dim3 grid(std::min(items, resident[f4]));
#ifdef ODO_TUNING
    if (!f4) {
        hipLaunchKernelGGL(k_knn2_mx, grid, dim3(256), 0, st, q, qn, q_stride, t, tn, t_stride, idx, dist, out_stride,
                           qlist, qcnt, ql_stride, npairs);
        return;
    }
#endif
    hipLaunchKernelGGL(k_knn2_f4, grid, dim3(256), 0, st, q, qn, q_stride, t, tn, t_stride, idx, dist, out_stride,
                       qlist, qcnt, ql_stride, npairs);
}
void launch_vo_lm(hipStream_t st, const float* xyz, const int* nkp, int kp_cap, int slot0, float th_depth_m,
                  uint32_t* lm_bits, int lm_words, int32_t* qlist, int* qcnt, int npairs) {
    int pw = 1;
    while (pw < kp_cap) pw <<= 1;
    const size_t lds = (size_t)pw * 8;
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)k_vo_lm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_vo_lm, dim3(npairs), dim3(PM_THREADS), lds, st, xyz, nkp, kp_cap, slot0, th_depth_m, lm_bits,
                       lm_words, qlist, qcnt);
}
void launch_pair_match(hipStream_t st, const int2* knn_idx, const int2* knn_dist, size_t knn_stride, const float* xyz,
                       const int* nkp, int kp_cap, int slot0, float ratio, const uint32_t* lm_bits, int lm_words,
                       int nsplit, size_t split_stride, int check_depth,
                       odo_dmatch* matches, int* n_matches, void* good, int* n_good, int32_t* f2_src,
                       uint64_t* sort_scratch, int match_cap, int npairs) {
    int pw = 1;
    while (pw < kp_cap || pw < match_cap) pw <<= 1;
    const size_t lds = psort_lds_bytes(pw);
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)k_pair_match, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_pair_match, dim3(npairs), dim3(PM_THREADS), lds, st, knn_idx, knn_dist, knn_stride, xyz, nkp,
                       kp_cap, slot0, ratio, lm_bits, lm_words, nsplit, split_stride, check_depth, matches, n_matches,
                       (SortEl*)good, n_good,
                       f2_src,
                       sort_scratch, match_cap);
}
// odo_debug_sort: the pair stage's std::sort on an arbitrary key array
__global__ void __launch_bounds__(PM_THREADS) k_sort_dbg(SortEl* __restrict__ a, int n, int pw) {
    extern __shared__ __attribute__((aligned(16))) uint64_t dyn_lds[];
    SortEl* A = reinterpret_cast<SortEl*>(dyn_lds);
    for (int i = threadIdx.x; i < n; i += PM_THREADS) A[i] = a[i];
    __syncthreads();
    block_gnu_sort(A, n, reinterpret_cast<uint8_t*>(dyn_lds) + (size_t)pw * 8,
                   *reinterpret_cast<PSortRanges*>(reinterpret_cast<uint8_t*>(dyn_lds) +
                                                  (((size_t)pw * 15 + 63) & ~(size_t)63)));
    for (int i = threadIdx.x; i < n; i += PM_THREADS) a[i] = A[i];
}

int launch_sort_dbg(hipStream_t st, void* a, int n) {
    int pw = 1;
    while (pw < n) pw <<= 1;
    const size_t lds = psort_lds_bytes(pw);
    if (lds > 160 * 1024) return -1;
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)k_sort_dbg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_sort_dbg, dim3(1), dim3(PM_THREADS), lds, st, (SortEl*)a, n, pw);
    return 0;
}

void launch_latch(hipStream_t st, double* latch, const void* good, const int* n_good, const int* n_matches,
                  const odo_dmatch* matches, const float* xyz, int kp_cap, int slot0, int npairs, int match_cap,
                  int min_inl, int sample_size, int iterations, const int* pair_valid, int* set_flag) {
    hipLaunchKernelGGL(k_latch, dim3(1), dim3(64), 0, st, latch, (const SortEl*)good, n_good, n_matches, matches, xyz,
                       kp_cap, slot0, npairs, match_cap, min_inl, sample_size, iterations, pair_valid, set_flag);
}
}  // namespace odo
