// Keypoint finalisation for gfx950: ORBextractor::operator()'s tail
// (Features/orbextractor.cpp:756-815) — IC_Angle (:14-39), computeOrbDescriptor
// (:43-85) on the Gaussian-blurred level, the level-0 scaling of the
// coordinates (:805-811) — and Frame::ExtractFeatures' per-keypoint geometry
// (Core/frame.cpp:139-164 UndistortKeyPoints / depth back-projection,
// :286-313).
//
//   k_finalize      16 lanes per keypoint, 4 keypoints per wave:
//                   IC angle from 9 aligned dwords per disc row (two rows per
//                   lane), realigned with alignbyte, bytes outside the disc
//                   masked, and the moments by udot4 (exact integers);
//                   rBRIEF with the rotation in packed fp32 and cvRound by the
//                   1.5*2^23 magic add, 32-bit gather offsets off the frame
//                   base, one ballot per test group
//   k_kp_geometry   one keypoint per lane: undistortion (5 double iterations)
//                   and the depth back-projection, shared with the ADAPTIVE
//                   extractor's finalisation (k_adaptive.hip)
#include "odo_device.h"
#include "odo_internal.h"
#ifndef ODO_EXTRACT_PRIO
#define ODO_EXTRACT_PRIO 0
#endif
#include "../../include/odo_orb_pattern.h"

namespace odo {

typedef float f32x2 __attribute__((ext_vector_type(2)));

__constant__ float4 c_patf[256];  // ORB_SLAM2 pattern test t: (x0, y0, x1, y1)
// the same tests as signed bytes, lane-major: c_pat8[s * 16 + w] = test w * 16 + s
// (k_finalize_lds lane s's sixteen tests in 64 contiguous bytes)
__constant__ uint32_t c_pat8[256];
#ifndef FIN_STAGE
#define FIN_STAGE 1  // k_finalize_lds's window staging: uniform-stride lane grid (1) or the chunk walk (0)
#endif
#ifndef FIN_PAT
#define FIN_PAT 2  // k_finalize_lds's pattern source: 0 c_patf, 1 an LDS copy of it, 2 c_pat8
#endif
__constant__ int c_umax16[16];    // IC_Angle disc half-widths per |v|

// 1.5 * 2^23: for |x| < 2^22, the float sum x + RND_MAGIC is x rounded half to
// even (cvRound) plus the magic, so its low mantissa bits are the integer.
#define RND_MAGIC 12582912.0f
#define RND_BITS 0x4B400000u

#ifndef FIN_WAVES_PER_EU
#define FIN_WAVES_PER_EU 1  // occupancy floor (launch bounds); 1 = compiler's choice
#endif
#define FIN_KPW 4              // keypoints per wave
#define FIN_KPB (4 * FIN_KPW)  // keypoints per workgroup
#ifdef ODO_TUNING  // retired per-lane-gather form (A/B only: the tuning build)
__global__ void __launch_bounds__(256, FIN_WAVES_PER_EU) k_finalize(const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                                                  size_t pyr_stride, const LevelDesc* __restrict__ lv, int nlevels,
                                                  const uint32_t* __restrict__ okp, const int* __restrict__ ocnt,
                                                  int okp_stride, orb_kp* __restrict__ kps, uint8_t* __restrict__ desc,
                                                  int* __restrict__ nkp, int kp_cap) {
    __shared__ uint64_t s_bal[4][16];
    __shared__ __attribute__((aligned(16))) uint32_t s_disc[16][8];  // byte masks of the disc rows |v| = 0..15
    if (threadIdx.x < 128) {
        const int av = threadIdx.x >> 3, i = threadIdx.x & 7;
        const int um = c_umax16[av];
        uint32_t m = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int u = 4 * i + bb - 15;  // dword i covers columns -15+4i .. -12+4i
            if (u >= -um && u <= um) m |= 0xffu << (8 * bb);
        }
        s_disc[av][i] = m;
    }
    // XCD-aware mapping: workgroups are dealt round-robin over the 8 XCDs, so
    // hardware id h runs on XCD h%8; logical ids are assigned so that each XCD
    // takes a contiguous run of (frame, keypoint-block) pairs and one frame's
    // pyramid and blurred levels are fetched into one L2 instead of eight.
    int bx = blockIdx.x, f = blockIdx.y;
    {
        const int total = gridDim.x * gridDim.y;
        if ((total & 7) == 0) {
            const int h = blockIdx.x + blockIdx.y * gridDim.x;
            const int lid = (h & 7) * (total >> 3) + (h >> 3);
            bx = lid % gridDim.x;
            f = lid / gridDim.x;
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, sub = lane & 15;  // keypoint slot in the wave, lane within it
    const int idx = bx * FIN_KPB + wave * FIN_KPW + g;
    // level lookup from per-level counts
    int lvl = -1, k = 0, acc = 0;
    for (int i = 0; i < nlevels; i++) {
        const int c = ocnt[f * nlevels + i];
        if (lvl < 0 && idx < acc + c) {
            lvl = i;
            k = idx - acc;
        }
        acc += c;
    }
    const int total = acc < kp_cap ? acc : kp_cap;
    if (bx == 0 && threadIdx.x == 0) nkp[f] = total;
    // a workgroup past the frame's last keypoint has nothing to do (the test is
    // uniform over the workgroup, so no barrier below is left waiting)
    if (bx * FIN_KPB >= total) return;
    const bool valid = lvl >= 0 && idx < kp_cap;
    // invalid slots run on a dummy in-level position and write nothing (no early
    // exit: the ballots and the barriers below need every wave)
    const LevelDesc L = lv[valid ? lvl : 0];
    const uint32_t key = valid ? okp[((size_t)f * nlevels + lvl) * okp_stride + k] : (16u | (16u << 12));
    const int kx = (int)(key & 0xfff) + 16, ky = (int)((key >> 12) & 0xfff) + 16;
    const float resp = (float)(key >> 24);
    // ---- IC_Angle: lane sub sums disc rows v0 = sub-15 and v1 = sub+1 (lanes
    // 0..14; lane 15's second row is masked to zero). Columns -15..16 of a row
    // are 8 dwords realigned from the 9 aligned dwords holding them (rows are
    // 16-byte aligned, a row's loads stay inside the pitch-padded level or the
    // pyramid's 64-byte tail). m10 = sum (u+16) I - 16 sum I, m01 = sum v I.
    int m10, m01;
    {
        const uint8_t* img = pyr + (size_t)f * pyr_stride + L.off;
        const bool has1 = sub < 15;
        const int v0 = sub - 15, v1 = has1 ? sub + 1 : 0;
        const int sh = (kx - 15) & 3;
        const uint32_t* r0 = reinterpret_cast<const uint32_t*>(img + (size_t)(ky + v0) * L.pitch + (kx - 15 - sh));
        const uint32_t* r1 = reinterpret_cast<const uint32_t*>(img + (size_t)(ky + v1) * L.pitch + (kx - 15 - sh));
        uint32_t w0[9], w1[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            w0[i] = r0[i];
            w1[i] = r1[i];
        }
        __syncthreads();  // s_disc
        const uint4* M0 = reinterpret_cast<const uint4*>(s_disc[-v0]);
        const uint4* M1 = reinterpret_cast<const uint4*>(s_disc[v1]);
        const uint4 a0 = M0[0], a1 = M0[1], b0 = M1[0], b1 = M1[1];
        const uint32_t z = has1 ? 0xffffffffu : 0u;
        const uint32_t mk0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const uint32_t mk1[8] = {b0.x & z, b0.y & z, b0.z & z, b0.w & z, b1.x & z, b1.y & z, b1.z & z, b1.w & z};
        uint32_t s0 = 0, s1 = 0, t = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t U = (uint32_t)(4 * i + 1) | ((uint32_t)(4 * i + 2) << 8) | ((uint32_t)(4 * i + 3) << 16) |
                               ((uint32_t)(4 * i + 4) << 24);
            const uint32_t d0 = __builtin_amdgcn_alignbyte(w0[i + 1], w0[i], sh) & mk0[i];
            const uint32_t d1 = __builtin_amdgcn_alignbyte(w1[i + 1], w1[i], sh) & mk1[i];
            s0 = __builtin_amdgcn_udot4(d0, 0x01010101u, s0, false);
            s1 = __builtin_amdgcn_udot4(d1, 0x01010101u, s1, false);
            t = __builtin_amdgcn_udot4(d0, U, t, false);
            t = __builtin_amdgcn_udot4(d1, U, t, false);
        }
        m10 = (int)t - 16 * (int)(s0 + s1);
        m01 = v0 * (int)s0 + v1 * (int)s1;
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
        m10 += __shfl_xor(m10, off);
        m01 += __shfl_xor(m01, off);
    }
    const float angle = fast_atan2((float)m01, (float)m10);
    // ---- rBRIEF: lane sub makes tests w*16+sub, w = 0..15. Per point
    // (x*b + y*a, x*a + (-y)*b) in packed fp32 — the reference's two products
    // and one sum per coordinate, each rounded once — then cvRound by the magic
    // add; offset = iy*pitch + ix in 32 bits with the magic folded into cofs.
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float ang = angle * factorPI;
    double sd, cd;
    sincos((double)ang, &sd, &cd);
    const float a = (float)cd, b = (float)sd;
    const f32x2 BA = {b, a}, AB = {a, b}, MAG = {RND_MAGIC, RND_MAGIC};
    const uint8_t* fb = blur + (size_t)f * pyr_stride;
    const uint32_t pitch = (uint32_t)L.pitch;
    // iy's low 24 bits are 0x400000 + dy (mul_u24), ix is RND_BITS + dx
    const uint32_t cofs = (uint32_t)L.off + (uint32_t)ky * pitch + (uint32_t)kx - 0x400000u * pitch - RND_BITS;
    int tv0[16], tv1[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const float4 P = c_patf[w * 16 + sub];
        f32x2 q0 = (f32x2){P.x, P.x} * BA + (f32x2){P.y, -P.y} * AB;
        f32x2 q1 = (f32x2){P.z, P.z} * BA + (f32x2){P.w, -P.w} * AB;
        q0 = q0 + MAG;
        q1 = q1 + MAG;
        const uint32_t o0 = __umul24(__float_as_uint(q0.x), pitch) + __float_as_uint(q0.y) + cofs;
        const uint32_t o1 = __umul24(__float_as_uint(q1.x), pitch) + __float_as_uint(q1.y) + cofs;
        tv0[w] = fb[o0];
        tv1[w] = fb[o1];
    }
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const uint64_t bal = __ballot(tv0[w] < tv1[w]);
        if (lane == 0) s_bal[wave][w] = bal;
    }
    __syncthreads();
    const int o = idx;
    if (valid && sub < 8) {
        // descriptor dword sub = tests 32*sub .. 32*sub+31 = groups 2sub, 2sub+1
        const uint32_t lo = (uint32_t)(s_bal[wave][2 * sub] >> (16 * g)) & 0xffffu;
        const uint32_t hi = (uint32_t)(s_bal[wave][2 * sub + 1] >> (16 * g)) & 0xffffu;
        reinterpret_cast<uint32_t*>(desc + ((size_t)f * kp_cap + o) * 32)[sub] = lo | (hi << 16);
    }
    if (valid && sub == 0) {
        orb_kp* kp = kps + (size_t)f * kp_cap + o;
        float px = (float)kx, py = (float)ky;
        if (lvl != 0) {
            px *= L.scale;
            py *= L.scale;
        }
        kp->x = px;
        kp->y = py;
        kp->size = (float)(int)(31 * L.scale);
        kp->angle = angle;
        kp->response = resp;
        kp->octave = lvl;
        kp->class_id = -1;
    }
}
#endif  // ODO_TUNING

// k_finalize_lds: the same finalisation with each keypoint's two patches
// staged in LDS by its 16 lanes with row-contiguous dword loads (the IC disc,
// rows ky-15..ky+15 of the level, 9 dwords each; the rBRIEF window, rows
// ky-18..ky+18 of the blurred level, 10 dwords each: rotated pattern points
// round into [-18, 18]). k_finalize's per-lane loads put the 16 lanes of a
// keypoint on 16 different rows, 64 cache lines per wave instruction through
// the texture path; staged, a wave instruction touches about two rows per
// keypoint, and the 512 rBRIEF samples become LDS byte reads.
#define FL_IC_W 9                    // dwords per staged IC row
#define FL_IC_N (31 * FL_IC_W)       // 279
#define FL_BR_W 10                   // dwords per staged rBRIEF row
#define FL_BR_N (37 * FL_BR_W)       // 370
// The rBRIEF window overwrites the IC disc once the angle is known (its loads
// are in flight since the start), so a keypoint holds 370 dwords of LDS
// instead of 649 and more workgroups fit a CU (round 2).
// dwords of LDS per keypoint, padded to 16 mod 32 (round 5): a wave's lanes
// 0-31 are two keypoints whose IC rows sit 9 dwords apart ({9s mod 32} for
// the 16 lanes: half the banks); the second keypoint 16 banks further takes
// exactly the other half ({16 + 9s}), where the unpadded 370 (18 mod 32)
// shared 14 of 16 banks with the first (PMC: 35.7 M conflict cycles, 1.4x
// the kernel's LDS cycles, round 4)
#define FL_KP_RAW FL_BR_N
#define FL_KP_DW (((FL_KP_RAW + 15) / 32) * 32 + 16)
template <int NW>  // waves (of 4 keypoints) per workgroup
__global__ void __launch_bounds__(64 * NW) k_finalize_lds(const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                                                      size_t pyr_stride, const LevelDesc* __restrict__ lv, int nlevels,
                                                      const uint32_t* __restrict__ okp, const int* __restrict__ ocnt,
                                                      int okp_stride, orb_kp* __restrict__ kps, uint8_t* __restrict__ desc,
                                                      int* __restrict__ nkp, int kp_cap) {
    if (ODO_EXTRACT_PRIO) __builtin_amdgcn_s_setprio(ODO_EXTRACT_PRIO);
#ifdef ODO_FINALIZE_PRIO
    __builtin_amdgcn_s_setprio(ODO_FINALIZE_PRIO);  // tuning: finalize's load chains ahead of co-runners
#endif
    __shared__ uint64_t s_bal[NW][16];
    // disc masks, rows padded to 12 dwords: the 16 lanes of a ds_read_b128
    // group read 16 different rows, which at 8 dwords met on 2 banks each
    __shared__ __attribute__((aligned(16))) uint32_t s_disc[16][12];
    __shared__ __attribute__((aligned(16))) uint32_t s_patch[NW * FIN_KPW][FL_KP_DW];
#if FIN_PAT == 1
    __shared__ float4 s_pat[256];
    for (int d = threadIdx.x; d < 256; d += 64 * NW) s_pat[d] = c_patf[d];
#endif
    for (int d = threadIdx.x; d < 128; d += 64 * NW) {
        const int av = d >> 3, i = d & 7;
        const int um = c_umax16[av];
        uint32_t m = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int u = 4 * i + bb - 15;
            if (u >= -um && u <= um) m |= 0xffu << (8 * bb);
        }
        s_disc[av][i] = m;
    }
    int bx = blockIdx.x, f = blockIdx.y;
    {
        const int total = gridDim.x * gridDim.y;
        if ((total & 7) == 0) {
            const int h = blockIdx.x + blockIdx.y * gridDim.x;
            const int lid = (h & 7) * (total >> 3) + (h >> 3);
            bx = lid % gridDim.x;
            f = lid / gridDim.x;
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, sub = lane & 15;
    const int kslot = wave * FIN_KPW + g;  // keypoint slot in the workgroup
    const int idx = bx * (NW * FIN_KPW) + kslot;
    int lvl = -1, k = 0, acc = 0;
    for (int i = 0; i < nlevels; i++) {
        const int c = ocnt[f * nlevels + i];
        if (lvl < 0 && idx < acc + c) {
            lvl = i;
            k = idx - acc;
        }
        acc += c;
    }
    const int total = acc < kp_cap ? acc : kp_cap;
    if (bx == 0 && threadIdx.x == 0) nkp[f] = total;
    if (bx * (NW * FIN_KPW) >= total) return;  // uniform over the workgroup
    const bool valid = lvl >= 0 && idx < kp_cap;
    const LevelDesc L = lv[valid ? lvl : 0];
    // an invalid slot stages and reads a dummy in-level patch and writes nothing
    const uint32_t key = valid ? okp[((size_t)f * nlevels + lvl) * okp_stride + k] : (16u | (16u << 12));
    const int kx = (int)(key & 0xfff) + 16, ky = (int)((key >> 12) & 0xfff) + 16;
    const float resp = (float)(key >> 24);
#if FIN_STAGE
    // Round 6: lanes sub < 15 as a fixed grid over each window's chunks —
    // the IC disc's 31 rows of 3 chunks (12 bytes) as 5 rows x 3 chunks per
    // step, the rBRIEF window's 37 rows of 5 chunks (8 bytes) as 3 rows x 5
    // chunks per step — so every step is one uniform address increment (5 or
    // 3 rows) instead of the wrap selects of the chunk walk below (7 + 13
    // loads instead of 6 + 12, ≈130 fewer VALU per wave); lane 15 and the
    // rows past a window's end load an in-window dummy and store nothing
    constexpr int IC_STEPS = 7, BR_STEPS = 13;
    uint2 vbr[BR_STEPS];  // the rBRIEF window's dwords (in flight during the IC angle)
    uint32_t* P = s_patch[kslot];
    const int sh = (kx - 15) & 3, sh2 = (kx - 18) & 3;
    const bool glane = sub < 15;
    const int ir = sub / 3, ic = sub - 3 * ir;  // IC: row in the step, chunk
    const int br = sub / 5, bc = sub - 5 * br;  // rBRIEF
    {
        const uint8_t* fpyr = pyr + (size_t)f * pyr_stride;
        const uint8_t* fblur = blur + (size_t)f * pyr_stride;
        const uint32_t pitch = (uint32_t)L.pitch;
        uint3 v[IC_STEPS];
        {
            const uint32_t o0 = (uint32_t)L.off + (uint32_t)(ky - 15) * pitch + (uint32_t)(kx - 15 - sh);
            uint32_t o = o0 + (uint32_t)ir * pitch + 12u * (uint32_t)ic;
#pragma unroll
            for (int j = 0; j < IC_STEPS; j++) {
                // rows ir + 5 j <= 30 for every lane (ir <= 5) until the last
                // step, which holds row 30 only (ir == 0)
                const bool ok = j + 1 < IC_STEPS || ir == 0;
                v[j] = *reinterpret_cast<const uint3*>(fpyr + (ok ? o : o0));
                o += 5u * pitch;
            }
        }
        {
            const uint32_t o0 = (uint32_t)L.off + (uint32_t)(ky - 18) * pitch + (uint32_t)(kx - 18 - sh2);
            uint32_t o = o0 + (uint32_t)br * pitch + 8u * (uint32_t)bc;
#pragma unroll
            for (int j = 0; j < BR_STEPS; j++) {
                // rows br + 3 j <= 36 for every lane (br <= 3) until the last
                // step, which holds row 36 only (br == 0)
                const bool ok = j + 1 < BR_STEPS || br == 0;
                vbr[j] = *reinterpret_cast<const uint2*>(fblur + (ok ? o : o0));
                o += 3u * pitch;
            }
        }
        {
            uint32_t* d = P + ir * FL_IC_W + 3 * ic;
#pragma unroll
            for (int j = 0; j < IC_STEPS; j++) {
                if (glane && (j + 1 < IC_STEPS || ir == 0)) {
                    d[0] = v[j].x;
                    d[1] = v[j].y;
                    d[2] = v[j].z;
                }
                d += 5 * FL_IC_W;
            }
        }
    }
#else
    uint2 vbr[12];  // the rBRIEF window's dwords (in flight during the IC angle)
    uint32_t* P = s_patch[kslot];
    const int sh = (kx - 15) & 3, sh2 = (kx - 18) & 3;
    {
        // Round 5: the windows as row chunks — the IC disc's 31 rows of 9
        // dwords as 93 chunks of 3 (global_load_dwordx3), the rBRIEF
        // window's 37 rows of 10 as 185 chunks of 2 (dwordx2) — chunk
        // sub + 16 j of the keypoint's 16 lanes. Until round 4 every lane
        // loaded single dwords: 42 load instructions per wave, and the
        // texture address / data units ran 93 % / 94 % busy for the whole
        // kernel (PMC, profiles/r05_l/pmcx_tex): 18 instructions now.
        // 32-bit byte offsets from the frame's base (uniform over the
        // workgroup: scalar base + vector offset loads); chunk rows and
        // columns stepped by 16 chunks without divisions (16 = 5 rows of 3
        // + 1, = 3 rows of 5 + 1); a lane past the end reloads the last chunk
        const uint8_t* fpyr = pyr + (size_t)f * pyr_stride;
        const uint8_t* fblur = blur + (size_t)f * pyr_stride;
        const uint32_t pitch = (uint32_t)L.pitch;
        uint3 v[6];
        {
            const uint32_t o0 = (uint32_t)L.off + (uint32_t)(ky - 15) * pitch + (uint32_t)(kx - 15 - sh);
            const uint32_t olast = o0 + 30u * pitch + 24u;
            int p = sub % 3;
            uint32_t o = o0 + (uint32_t)(sub / 3) * pitch + 12u * (uint32_t)p;
#pragma unroll
            for (int j = 0; j < 6; j++) {
                v[j] = *reinterpret_cast<const uint3*>(fpyr + (sub + 16 * j < 93 ? o : olast));
                const bool wrap = p == 2;
                o += wrap ? 6u * pitch - 24u : 5u * pitch + 12u;
                p = wrap ? 0 : p + 1;
            }
        }
        {
            const uint32_t o0 = (uint32_t)L.off + (uint32_t)(ky - 18) * pitch + (uint32_t)(kx - 18 - sh2);
            const uint32_t olast = o0 + 36u * pitch + 32u;
            int p = sub % 5;
            uint32_t o = o0 + (uint32_t)(sub / 5) * pitch + 8u * (uint32_t)p;
#pragma unroll
            for (int j = 0; j < 12; j++) {
                vbr[j] = *reinterpret_cast<const uint2*>(fblur + (sub + 16 * j < 185 ? o : olast));
                const bool wrap = p == 4;
                o += wrap ? 4u * pitch - 32u : 3u * pitch + 8u;
                p = wrap ? 0 : p + 1;
            }
        }
        // IC chunk c = sub + 16 j: row c / 3, dwords 3 (c % 3) .. + 2 of it
        {
            int r = sub / 3, p = sub % 3;
#pragma unroll
            for (int j = 0; j < 6; j++) {
                if (sub + 16 * j < 93) {
                    uint32_t* d = P + r * FL_IC_W + 3 * p;
                    d[0] = v[j].x;
                    d[1] = v[j].y;
                    d[2] = v[j].z;
                }
                const bool wrap = p == 2;
                r += wrap ? 6 : 5;
                p = wrap ? 0 : p + 1;
            }
        }
    }
#endif
    __syncthreads();  // s_disc, the patches
    int m10, m01;
    {
        const bool has1 = sub < 15;
        const int v0 = sub - 15, v1 = has1 ? sub + 1 : 0;
        const uint32_t* r0 = P + (v0 + 15) * FL_IC_W;
        const uint32_t* r1 = P + (v1 + 15) * FL_IC_W;
        uint32_t w0[9], w1[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            w0[i] = r0[i];
            w1[i] = r1[i];
        }
        const uint4* M0 = reinterpret_cast<const uint4*>(s_disc[-v0]);
        const uint4* M1 = reinterpret_cast<const uint4*>(s_disc[v1]);
        const uint4 a0 = M0[0], a1 = M0[1], b0 = M1[0], b1 = M1[1];
        const uint32_t z = has1 ? 0xffffffffu : 0u;
        const uint32_t mk0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const uint32_t mk1[8] = {b0.x & z, b0.y & z, b0.z & z, b0.w & z, b1.x & z, b1.y & z, b1.z & z, b1.w & z};
        uint32_t s0 = 0, s1 = 0, t = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t U = (uint32_t)(4 * i + 1) | ((uint32_t)(4 * i + 2) << 8) | ((uint32_t)(4 * i + 3) << 16) |
                               ((uint32_t)(4 * i + 4) << 24);
            const uint32_t d0 = __builtin_amdgcn_alignbyte(w0[i + 1], w0[i], sh) & mk0[i];
            const uint32_t d1 = __builtin_amdgcn_alignbyte(w1[i + 1], w1[i], sh) & mk1[i];
            s0 = __builtin_amdgcn_udot4(d0, 0x01010101u, s0, false);
            s1 = __builtin_amdgcn_udot4(d1, 0x01010101u, s1, false);
            t = __builtin_amdgcn_udot4(d0, U, t, false);
            t = __builtin_amdgcn_udot4(d1, U, t, false);
        }
        m10 = (int)t - 16 * (int)(s0 + s1);
        m01 = v0 * (int)s0 + v1 * (int)s1;
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
        m10 += __shfl_xor(m10, off);
        m01 += __shfl_xor(m01, off);
    }
    const float angle = fast_atan2((float)m01, (float)m10);
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float ang = angle * factorPI;
    double sd, cd;
    sincos((double)ang, &sd, &cd);
    const float a = (float)cd, b = (float)sd;
    const f32x2 BA = {b, a}, AB = {a, b}, MAG = {RND_MAGIC, RND_MAGIC};
    // staged byte of rotated offset (iy, ix): (iy + 18) * 40 + ix + 18 + sh2; the
    // magic-rounded floats carry RND_BITS + offset in their bits
    __syncthreads();  // every IC disc read
#if FIN_STAGE
    {
        uint32_t* d = P + br * FL_BR_W + 2 * bc;
#pragma unroll
        for (int j = 0; j < BR_STEPS; j++) {
            if (glane && (j + 1 < BR_STEPS || br == 0)) *reinterpret_cast<uint2*>(d) = vbr[j];
            d += 3 * FL_BR_W;
        }
    }
#else
    {
        // rBRIEF chunk c = sub + 16 j: row c / 5, dwords 2 (c % 5), + 1
        int r = sub / 5, p = sub % 5;
#pragma unroll
        for (int j = 0; j < 12; j++) {
            if (sub + 16 * j < 185) *reinterpret_cast<uint2*>(P + r * FL_BR_W + 2 * p) = vbr[j];
            const bool wrap = p == 4;
            r += wrap ? 4 : 3;
            p = wrap ? 0 : p + 1;
        }
    }
#endif
    __syncthreads();
    const uint8_t* PB = reinterpret_cast<const uint8_t*>(P);
    // iy's low 24 bits are 0x400000 + dy (a 24-bit multiply: v_mad_u32_u24,
    // full rate, where the 32-bit product took v_mad_u64_u32 until round 5)
    const uint32_t cofs = (uint32_t)(18 * 4 * FL_BR_W + 18 + sh2) - 0x400000u * (uint32_t)(4 * FL_BR_W) - RND_BITS;  // mod 2^32
    int tv0[16], tv1[16];
#if FIN_PAT == 2
    uint32_t pat8[16];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint4 q = reinterpret_cast<const uint4*>(c_pat8)[sub * 4 + u];
        pat8[4 * u] = q.x, pat8[4 * u + 1] = q.y, pat8[4 * u + 2] = q.z, pat8[4 * u + 3] = q.w;
    }
#endif
#pragma unroll
    for (int w = 0; w < 16; w++) {
#if FIN_PAT == 2
        const uint32_t pw = pat8[w];
        const float4 Pt = {(float)(int8_t)(pw & 0xff), (float)(int8_t)((pw >> 8) & 0xff),
                           (float)(int8_t)((pw >> 16) & 0xff), (float)(int8_t)(pw >> 24)};
#elif FIN_PAT == 1
        const float4 Pt = s_pat[w * 16 + sub];
#else
        const float4 Pt = c_patf[w * 16 + sub];
#endif
        f32x2 q0 = (f32x2){Pt.x, Pt.x} * BA + (f32x2){Pt.y, -Pt.y} * AB;
        f32x2 q1 = (f32x2){Pt.z, Pt.z} * BA + (f32x2){Pt.w, -Pt.w} * AB;
        q0 = q0 + MAG;
        q1 = q1 + MAG;
        const uint32_t o0 = __umul24(__float_as_uint(q0.x), (uint32_t)(4 * FL_BR_W)) + __float_as_uint(q0.y) + cofs;
        const uint32_t o1 = __umul24(__float_as_uint(q1.x), (uint32_t)(4 * FL_BR_W)) + __float_as_uint(q1.y) + cofs;
        tv0[w] = PB[o0];
        tv1[w] = PB[o1];
    }
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const uint64_t bal = __ballot(tv0[w] < tv1[w]);
        if (lane == 0) s_bal[wave][w] = bal;
    }
    __syncthreads();
    const int o = idx;
    if (valid && sub < 8) {
        const uint32_t lo = (uint32_t)(s_bal[wave][2 * sub] >> (16 * g)) & 0xffffu;
        const uint32_t hi = (uint32_t)(s_bal[wave][2 * sub + 1] >> (16 * g)) & 0xffffu;
        reinterpret_cast<uint32_t*>(desc + ((size_t)f * kp_cap + o) * 32)[sub] = lo | (hi << 16);
    }
    if (valid && sub == 0) {
        orb_kp* kp = kps + (size_t)f * kp_cap + o;
        float px = (float)kx, py = (float)ky;
        if (lvl != 0) {
            px *= L.scale;
            py *= L.scale;
        }
        kp->x = px;
        kp->y = py;
        kp->size = (float)(int)(31 * L.scale);
        kp->angle = angle;
        kp->response = resp;
        kp->octave = lvl;
        kp->class_id = -1;
    }
}

// UndistortKeyPoints + depth back-projection (frame.cpp:139-164, 286-313) of
// every finalised keypoint, one per lane.
__global__ void __launch_bounds__(256) k_kp_geometry(const orb_kp* __restrict__ kps, const int* __restrict__ nkp,
                                                     const uint16_t* __restrict__ depth, size_t depth_stride, int img_w,
                                                     FrameCalib cal, float* __restrict__ kun, float* __restrict__ xyz,
                                                     float* __restrict__ ur, int kp_cap) {
    const int f = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkp[f]) return;
    const size_t o = (size_t)f * kp_cap + i;
    const float2 p = *reinterpret_cast<const float2*>(&kps[o].x);
    kp_geometry(p.x, p.y, cal, depth + (size_t)f * depth_stride, img_w, kun + o * 2, xyz + o * 3, ur + o);
}

void upload_finalize_constants() {
    float4 pat[256];
    for (int t = 0; t < 256; t++)
        pat[t] = make_float4((float)ODO_ORB_PATTERN[4 * t], (float)ODO_ORB_PATTERN[4 * t + 1],
                             (float)ODO_ORB_PATTERN[4 * t + 2], (float)ODO_ORB_PATTERN[4 * t + 3]);
    hipMemcpyToSymbol(HIP_SYMBOL(c_patf), pat, sizeof(pat));
    uint32_t pat8[256];
    for (int sl = 0; sl < 16; sl++)
        for (int w = 0; w < 16; w++) {
            const int t = w * 16 + sl;
            uint32_t v = 0;
            for (int i = 0; i < 4; i++) v |= (uint32_t)(uint8_t)(int8_t)ODO_ORB_PATTERN[4 * t + i] << (8 * i);
            pat8[sl * 16 + w] = v;
        }
    hipMemcpyToSymbol(HIP_SYMBOL(c_pat8), pat8, sizeof(pat8));
    const int umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
    hipMemcpyToSymbol(HIP_SYMBOL(c_umax16), umax, sizeof(umax));
}

void launch_kp_geometry(hipStream_t st, const orb_kp* kps, const int* nkp, const uint16_t* depth, size_t depth_stride,
                        int img_w, FrameCalib cal, float* kun, float* xyz, float* ur, int kp_cap, int nframes) {
    dim3 g((kp_cap + 255) / 256, nframes);
    hipLaunchKernelGGL(k_kp_geometry, g, dim3(256), 0, st, kps, nkp, depth, depth_stride, img_w, cal, kun, xyz, ur,
                       kp_cap);
}

void launch_finalize(hipStream_t st, const uint8_t* pyr, const uint8_t* blur, size_t pyr_stride, const LevelDesc* lv,
                     int nlevels, const uint32_t* okp, const int* ocnt, int okp_stride, const uint16_t* depth,
                     size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps, uint8_t* desc, float* kun, float* xyz,
                     float* ur, int* nkp, int kp_cap, int nframes, bool geometry) {
    dim3 g((kp_cap + FIN_KPB - 1) / FIN_KPB, nframes);
    // ODO_FIN_LDS: 0 the per-lane-gather k_finalize; 1 the staged kernel at 4
    // waves (16 keypoints, 42.5 KB LDS) per workgroup; 2 (default) at 2 waves
    // (8 keypoints, 21 KB: more workgroups resident per CU); 3 at 1 wave
    static const int staged = [] {
        const char* e = odo_knob("ODO_FIN_LDS");
        return e ? atoi(e) : 2;
    }();
#ifdef ODO_TUNING
    if (staged == 3)  // one wave (4 keypoints, 6.3 KB) per workgroup
        hipLaunchKernelGGL(k_finalize_lds<1>, dim3((kp_cap + 3) / 4, nframes), dim3(64), 0, st, pyr, blur, pyr_stride,
                           lv, nlevels, okp, ocnt, okp_stride, kps, desc, nkp, kp_cap);
    else if (staged == 1)
        hipLaunchKernelGGL(k_finalize_lds<4>, g, dim3(256), 0, st, pyr, blur, pyr_stride, lv, nlevels, okp, ocnt,
                           okp_stride, kps, desc, nkp, kp_cap);
    else if (staged == 0)
        hipLaunchKernelGGL(k_finalize, g, dim3(256), 0, st, pyr, blur, pyr_stride, lv, nlevels, okp, ocnt, okp_stride,
                           kps, desc, nkp, kp_cap);
    else
#endif
        hipLaunchKernelGGL(k_finalize_lds<2>, dim3((kp_cap + 7) / 8, nframes), dim3(128), 0, st, pyr, blur, pyr_stride,
                           lv, nlevels, okp, ocnt, okp_stride, kps, desc, nkp, kp_cap);
    if (geometry) launch_kp_geometry(st, kps, nkp, depth, depth_stride, img_w, cal, kun, xyz, ur, kp_cap, nframes);
}

}  // namespace odo
