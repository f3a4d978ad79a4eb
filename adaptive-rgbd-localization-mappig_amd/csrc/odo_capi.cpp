// Host orchestration and C-ABI (include/odo.h) of the MI355X odometry path.
//
// A context owns all HBM scratch sized for max_batch frames, the per-image-size
// geometry tables (pyramid levels, FAST cells, resize coefficients) and the
// cross-frame state the reference keeps in globals: the previous frame
// (Tracking::mpLastFrame) and the DepthCovariance latch.
//
// Batches are pipelined over two streams. The extraction stream rolls the
// previous batch's last frame into slot 0 of a frame set and extracts the new
// frames into slots 1..n; the pair stream then matches, runs RANSAC and PnP on
// that set. Frame sets (and the RANSAC scratch) alternate between batches, so
// batch k+1's throughput-bound extraction overlaps batch k's latency-bound
// pair stages; per-set events order the reuse (set s is rewritten only after
// the pair stages of batch k-1 that read it have finished).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <mutex>

#include "../../include/odo.h"
#include "odo_device.h"
#include "odo_internal.h"

using namespace odo;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) return fail(ODO_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

inline int cvRoundH(float v) { return (int)lrintf(v); }
inline int cvFloorH(float v) {
    int i = (int)v;
    return i - (i > v);
}
inline int satShort(float v) {
    int r = cvRoundH(v);
    return std::min(std::max(r, -32768), 32767);
}

template <typename T>
int dalloc(T** p, size_t count) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) return fail(ODO_ERR_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
    return ODO_OK;
}

uint32_t splitmix_host(uint64_t base, uint64_t pair) { return pair_seed(base, pair); }

}  // namespace

// Device scratch of the per-stage entry points (odo_extract ... odo_kabsch):
// owned by a context, bump-allocated per call, grown on demand and never freed
// per call. A call that outgrows the block takes an extra block; the next call
// replaces the blocks by one of their total size. Every allocation is checked
// (a failed one sets `failed`, which the entry point turns into
// ODO_ERR_DEVICE). begin() may hipFree the blocks: its callers first make sure
// that no kernel of an earlier call still uses them (the per-stage entry
// points are synchronous; hypotheses mode, whose _dev / _finish calls queue
// kernels asynchronously, synchronises its stream before begin()).
struct DevArena {
    std::vector<std::pair<uint8_t*, size_t>> blocks;
    size_t used = 0;
    bool failed = false;
    ~DevArena() { release(); }
    void release() {
        for (auto& b : blocks) (void)hipFree(b.first);
        blocks.clear();
        used = 0;
    }
    void begin() {
        failed = false;
        if (blocks.size() > 1) {
            size_t tot = 0;
            for (auto& b : blocks) tot += b.second;
            release();
            grow(tot);
        }
        used = 0;
    }
    bool grow(size_t bytes) {
        uint8_t* p = nullptr;
        if (hipMalloc((void**)&p, bytes) != hipSuccess) {
            failed = true;
            return false;
        }
        blocks.push_back({p, bytes});
        used = 0;
        return true;
    }
    void* take(size_t bytes) {
        bytes = std::max<size_t>((bytes + 255) & ~(size_t)255, 256);
        if (blocks.empty() || used + bytes > blocks.back().second)
            if (!grow(std::max(bytes, blocks.empty() ? (size_t)16 << 20 : blocks.back().second))) return nullptr;
        void* r = blocks.back().first + used;
        used += bytes;
        return r;
    }
};

// Frame sets in flight (4): batch k extracts into set k%NSETS while the pair and
// PnP stages of batches k-1 and k-2 still read theirs, so the extraction
// stream never waits on the PnP latency of the batch just before it.
#ifndef ODO_EVFENCE
#define ODO_EVFENCE 1  // stream-ordering events: 0 default (system-scope fence), 1 no system fence, 2 device-scope release
#endif
#define ODO_SYNC_EVENT_FLAGS \
    (hipEventDisableTiming | (ODO_EVFENCE == 1 ? hipEventDisableSystemFence : ODO_EVFENCE == 2 ? hipEventReleaseToDevice : 0u))
#ifndef KNN_GATE
#define KNN_GATE 0
#endif
#ifndef PYR_WAIT
#define PYR_WAIT 3  // measured: 1.921-1.938 vs 1.933-1.989 ms per step, hard workload unchanged (profiles/r05_q)
#endif
#ifndef ODO_NSETS
#define ODO_NSETS 4  // measured: 4 sets 60.1k vs 3 sets 57.7k frames/s (256-frame batches)
#endif
constexpr int NSETS = ODO_NSETS;
// batch b - PYR_WAIT must not share batch b's frame set: its PnP events are
// re-recorded by batch b - PYR_WAIT + NSETS
static_assert(PYR_WAIT >= 0 && PYR_WAIT < ODO_NSETS, "PYR_WAIT must be below ODO_NSETS");
// output rows per resize workgroup
constexpr int RZ_RB = 16;

struct HypSession;  // hypotheses-mode RANSAC state (odo_ransac_hyps .. _finish)
static void free_hyp_session(HypSession* h);

struct odo_ctx {
    odo_config cfg{};
    HypSession* hs = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;   // extraction
    hipStream_t pstream = nullptr;  // pair stages
    hipStream_t pstream2 = nullptr;  // pair stages of odd batches (schedule 5)
    hipStream_t pstream3 = nullptr;  // third pair stream (schedule 5, ODO_PSTREAMS=3)
    int npstreams = 2;
    bool knn_pair = true;  // schedule 5 (ODO_KNN_PAIR=0: on the extraction stream): kNN-2 at the head of the pair stream, 88.2k vs 86.5k frames/s (kNN roofline 0.85 vs 0.90)
    hipStream_t cur_p = nullptr;     // pair stream of the batch being queued
    // KNN_GATE / ODO_KNN_GATE (tuning): the next batch's extraction waits
    // for this batch's kNN-2 (no pyramid / kNN-2 overlap)
    bool knn_gate = KNN_GATE != 0;
    // the extraction of batch b waits for the PnP of batch b - pyr_wait (0:
    // not), so the pyramid does not share the CUs with a PnP / RANSAC
    // evaluation still running from an earlier batch (PYR_WAIT; ODO_PYR_WAIT)
    int pyr_wait = PYR_WAIT;
    int batch_set[8] = {};  // set of batch b at [b & 7]
    hipEvent_t ev_knn = nullptr;
    bool knn_rec = false;
    std::vector<hipStream_t> owned;  // streams created (the rest alias them)
    hipEvent_t ev_latch = nullptr;   // after the last queued k_latch (schedule 5)
    bool latch_rec = false;
    bool latched = false;  // this batch leaves the latch kernel out (see run_pairs)
    // ODO_GEO_PAIR: this batch's geometry and roll are on its pair stream;
    // ev_geo[set] follows the set's geometry kernel (the next batch's roll
    // reads the last frame's kun / xyz / uR); host_call: a track_host
    // batch (its depth reads must stay on the extraction stream)
    bool geo_pair = false, host_call = false;
    // ODO_EARLY_WAIT (run_extract): the next batch's extraction-stream waits
    // were queued during this one (pre_waited = that batch's counter)
    bool early_waits = false;
    bool defer_pdone = false;  // odo_track_batch_async: PnP-done events after the result copy
    uint64_t pre_waited = ~(uint64_t)0;
    hipEvent_t ev_geo[NSETS] = {};
    bool geo_rec[NSETS] = {};
    uint64_t batch_counter = 0;
    int W = 0, H = 0, maxb = 0, slots = 0, nlevels = 0;
    std::vector<LevelDesc> lv_h;
    std::vector<CellDesc> cells_h;
    std::vector<int> rx_off, ry_off, rz_rows;
    // k_pyramid (gray + levels, and the blurred levels) where its host checks
    // pass (pyramid_fusable, pyramid_blur_fusable) and odo_kernel_forms.pyramid
    // asks for it: ODO_PYRAMID_FORM_AUTO takes it for batches of at least
    // PYR_FUSED_MIN_FRAMES frames (a workgroup per frame: a small batch would
    // leave most CUs idle, one frame takes 0.45 vs 0.28 ms)
    int pform = ODO_PYRAMID_FORM_AUTO;
    bool pyr_fusable = false, blur_fusable = false;
    LevelDesc* lv = nullptr;
    CellDesc* cells = nullptr;
    ResizeX* rx = nullptr;
    ResizeY* ry = nullptr;
    std::vector<ResizeY> ry_h;  // host copy (k_pyramid's split plan)
    int ncells = 0, cell_cap = 0, kp_cap = 0, okp_stride = 0, node_cap = 0, match_cap = 0, mask_words = 0;
    int max_blur_tiles = 0;
    int fast_roi = 0;  // largest FAST cell ROI side
    std::vector<FastSeg> fsegs_h;  // k_fast_seg's segments (cell-row runs)
    FastSeg* fsegs = nullptr;
    FastLds fs_lds{};
    size_t pyr_size = 0, keys_per_frame = 0;
    FrameCalib cal{};
    RansacCfg rcfg{};
    // frame buffers ([2 sets][slots])
    uint8_t *pyr = nullptr, *blur = nullptr;
    uint32_t* cand = nullptr;
    int* cand_cnt = nullptr;
    uint32_t* keys = nullptr;
    int32_t* knode = nullptr;
    uint8_t* kquad = nullptr;
    uint32_t* okp = nullptr;
    int* ocnt = nullptr;
    orb_kp* kps = nullptr;
    uint8_t* desc = nullptr;
    float *kun = nullptr, *xyz = nullptr, *ur = nullptr;
    int* nkp = nullptr;
    // staging for host inputs: two device buffers of max_batch frames each,
    // filled on the copy stream (odo_track_batch_host) while the extraction
    // stream reads the other one
    uint8_t* bgr_in[2] = {};
    uint16_t* depth_in[2] = {};
    hipStream_t cstream = nullptr;                      // H2D copies of host inputs
    hipEvent_t ev_in_copied[2] = {}, ev_in_free[2] = {};
    bool in_used[2] = {};
    // the last odo_track_batch_host_sparse_depth batch's depth reads (extraction
    // stream): the caller's depth buffer is in use until this event
    hipEvent_t ev_depth_done = nullptr;
    bool depth_busy = false;
    // page-locked staging of the per-stage (synchronous) entry points: their
    // inputs are packed here and uploaded with one DMA, their outputs come
    // back here with async copies into pinned memory and one sync
    uint8_t* stage_h = nullptr;
    size_t stage_cap = 0;
    // hypotheses mode (odo_ransac_hyps*): device scratch kept across sessions
    // (grow-only: a session per pair used to hipMalloc / hipFree its own,
    // 0.5 ms of the 1.2 ms per pair of round 4) and the session's packed
    // inputs in page-locked memory (one DMA), reused once hyp_up has passed
    DevArena hyp_arena;
    uint8_t* hyp_stage_h = nullptr;
    size_t hyp_stage_cap = 0;
    hipEvent_t hyp_up = nullptr;
    bool hyp_up_rec = false;
    int in_next = 0;
    // pair buffers ([maxb])
    int2 *knn_idx[NSETS] = {}, *knn_dist[NSETS] = {};  // per frame set
    // per frame set: the query frames' VO-landmark bits and kNN-2 query lists
    uint32_t* lm_bits[NSETS] = {};
    int32_t* qlist[NSETS] = {};
    int* qcnt[NSETS] = {};
    int lm_words = 0;
    int knn_split = 2;  // kNN-2 train splits per query block (ODO_KNN_SPLIT): more waves for short query lists
    // kNN-2 form (ODO_KNN_MFMA): 0 the VALU xor/popcount kernel k_knn2, 1 exact
    // int8 sign-vector products on the matrix cores (k_knn2_mx), 2 the same on
    // FP4 (e2m1 +-1) operands (k_knn2_f4, the default: 97 us vs 137-150 us for
    // the 256-pair bench launch alone)
    int knn_mx = KNN_FMT_F4;
    int last_knn_set = -1, last_knn_n = 0;  // the most recent batch's kNN-2 launch (odo_knn_replay_time)
    uint64_t* sort_scratch = nullptr;
    double* latch = nullptr;
    void* rscr[NSETS] = {};  // RANSAC scratch per frame set
    uint32_t* masks = nullptr;
    // per frame set: the pair stages of batch k write set k%NSETS while the
    // PnP launches of batches k-1, k-2 may still read their own sets
    struct PairBufs {
        odo_dmatch* matches = nullptr;
        int *n_matches = nullptr, *n_good = nullptr, *pair_valid = nullptr;
        void* good = nullptr;  // SortEl
        int32_t* f2_src = nullptr;
        uint32_t* best_mask = nullptr;
        odo_pair_result* res = nullptr;
        float* T12 = nullptr;
        void* edges = nullptr;
        uint8_t* pnp_mask = nullptr;
        int* pair_phase = nullptr;  // per pair: finished by RANSAC part 1
    } pb[NSETS];
    // sequence state: the last tracked batch sits in frame set seq_set (its
    // last frame at slot seq_n); getters read view_set / view_n
    bool has_prev = false;
    uint64_t pair_counter = 0;
    int seq_set = NSETS - 1, seq_n = 0;
    int view_set = 0, last_n = 0;
    std::vector<int> valid_h;
    hipEvent_t ev[16];
    int nev = 0;
    hipStream_t side = nullptr;  // RANSAC rand() words, ahead of the pair stages
    hipStream_t pnpa = nullptr;  // PnP of the pairs RANSAC part 1 finished
    hipStream_t pnpb = nullptr;  // PnP of the pairs RANSAC part 2 finished
    hipEvent_t ev_xdone[NSETS] = {}, ev_raw[NSETS] = {};
    // schedule 5 with ODO_BLUR_STREAM=1: the pyramid blur of a batch runs on
    // its own stream beside FAST + octree, joined before finalize (measured
    // 76.2 k vs 77.7 k frames/s without: the CUs are already shared with the
    // pair streams, so it stays off by default)
    hipStream_t bstream = nullptr;
    hipEvent_t ev_pyr[NSETS] = {}, ev_blur[NSETS] = {};
    // per set: RANSAC part 1 / part 2 done, PnP A / PnP B done
    hipEvent_t ev_ra[NSETS] = {}, ev_rb[NSETS] = {}, ev_pa[NSETS] = {}, ev_pb[NSETS] = {};
    bool pdone_rec[NSETS] = {};
    hipStream_t pdone_st[NSETS] = {};  // the stream that last recorded ev_pa / ev_pb of a set
    bool serial = false;
    bool timing = false;
    // stream layout (ODO_SCHED). Only the streams a schedule uses are created:
    // every stream beyond the process's GPU_MAX_HW_QUEUES (4) hardware queues
    // shares one with another stream and serialises behind it.
    // 5 (default) = extraction (+ kNN-2) | two pair streams taking alternate
    //     batches, each running its batch's rand() words, match, RANSAC and
    //     PnP, so one batch's long RANSAC/PnP overlaps the next batch's pair
    //     stages (the DepthCovariance latch kernels are ordered by an event):
    //     52.9k frames/s at 128-frame batches;
    // 2 = extraction | side (words) | pair stages | one PnP stream: 42.1k;
    // 1 = as 2 with two PnP launches on two streams: 41.9k;
    // 0 = words on the extraction stream; 3 = kNN-2 + words on the side
    //     stream; 4 = words at the head of the pair stream.
    int sched = 5;
    // ODO_SKIP (measurement only; results are invalid when set): bit 0 skips
    // the PnP launches, bit 1 RANSAC part 2, bit 2 every pair stage, bit 3 kNN-2,
    // bit 4 RANSAC (schedule 2)
    int skip = 0;
    // ADAPTIVE grid extractor (ODO_DETECTOR_ADAPTIVE_FAST): cell / band
    // tables and per-batch scratch (extraction stream only), plus the
    // persistent per-cell DetectorAdjuster thresholds
    bool adaptive = false;
    int ad_ncells = 0, ad_nbands = 0, ad_mpc = 0;
    std::vector<AdCell> adc_h;
    std::vector<AdBand> adb_h;
    AdCell* adc = nullptr;
    AdBand* adb = nullptr;
    uint8_t* smap = nullptr;
    size_t smap_stride = 0, acand_stride = 0, abig_stride = 0;
    uint32_t *acand = nullptr, *abig = nullptr, *acell = nullptr, *akp = nullptr;
    int *aband_cnt = nullptr, *ahist = nullptr, *atsel = nullptr, *ansel = nullptr, *acell_cnt = nullptr;
    double* athresh = nullptr;
    float a_cos = 1.f, a_sin = 0.f;
    // ODO_DETECTOR_ADAPTIVE_ORB (k_adaptive_orb.hip): cell-level images, bands,
    // S-map tiles; per-batch cell pyramids / S maps / survivors / selection
    // scratch (extraction stream only); the frame pyramid and its blur come
    // from pyr / blur
    bool adaptive_orb = false;
    std::vector<OaImg> oai_h;
    std::vector<OaCell> oac_h;
    std::vector<OaBand> oab_h;
    OaImg* oai = nullptr;
    OaCell* oac = nullptr;
    OaBand* oab = nullptr;
    OaScales osc{};
    int oa_ncap = 0, oa_buf0 = 0, oa_buf1 = 0, oa_maxpitch = 16;
    size_t cp_stride = 0, ocand_stride = 0, oscr_stride = 0;
    uint8_t *cpyr = nullptr, *oscr = nullptr;
    uint32_t* ocand = nullptr;
    int *oband_cnt = nullptr, *ohist = nullptr, *ophist = nullptr;
    uint64_t *ocell = nullptr, *oakp = nullptr;
    DevArena arena;  // per-stage entry points' device scratch
    int* h_open = nullptr;  // page-locked [NSETS]: RANSAC open pairs of the last batch per set (launch hint)
    // page-locked, host-coherent: k_latch writes 1 once the latch holds a
    // value; with ev_latch complete the host then stops ordering (and
    // launching) the no-op latch kernels of later batches
    int* latch_set_h = nullptr;
    // Hamming-match kernel timing (odo_set_timing mode 2): an event pair
    // around the kNN-2 launch of every batch, read back and summed lazily
    static constexpr int KT_RING = 256;
    bool ktiming = false;
    hipEvent_t kt0[KT_RING] = {}, kt1[KT_RING] = {};
    int kt_next = 0, kt_pending = 0;
    double kt_sum_ms = 0;
    long kt_count = 0;
    // per-step marks (odo_step_marks): every collected kNN-2 start as ms after
    // kt_ref, an event recorded when mode 2 was set
    hipEvent_t kt_ref = nullptr;
    std::vector<double> kt_marks;
};

static inline size_t fbase(const odo_ctx* c, int set) { return (size_t)set * c->slots; }
// the set the next batch extracts into
static inline int next_set(const odo_ctx* c) { return (c->seq_set + 1) % NSETS; }

#ifndef ODO_WAIT_DEDUP
#define ODO_WAIT_DEDUP 1
#endif
#ifndef ODO_EARLY_WAIT
#define ODO_EARLY_WAIT 0
#endif
#ifndef ODO_GEO_PAIR
// schedule 5, device inputs: the keypoint geometry (undistort, depth) and the
// slot-0 roll run at the head of the batch's pair stream instead of at the
// end of the extraction stream, the step's critical path (round 6: 152.0-152.6
// vs 150.9-151.3 k frames/s, three alternations on one box, profiles/r06_d)
#define ODO_GEO_PAIR 1
#endif
// `st` waits until the PnP launches (and, async, the result copy) of the batch
// that last used frame set `set` are done. Every wait is a barrier packet the
// queue processes in order: schedule 5 records ev_pa and ev_pb at the same
// point of one stream, so one of them is enough, and none is needed on that
// stream itself (ODO_WAIT_DEDUP; 0 = the round-5 waits on both events).
static int wait_pnp_done(odo_ctx* c, hipStream_t st, int set) {
    if (ODO_WAIT_DEDUP && c->sched == 5) {
        if (st != c->pdone_st[set]) HIPCHK(hipStreamWaitEvent(st, c->ev_pb[set], 0));
        return ODO_OK;
    }
    HIPCHK(hipStreamWaitEvent(st, c->ev_pa[set], 0));
    HIPCHK(hipStreamWaitEvent(st, c->ev_pb[set], 0));
    return ODO_OK;
}

// The extraction stream's waits before batch number `bc` (the batch_counter it
// will have): its frame set is free once the PnP of the batch that last used
// it is done, and (schedule 5) the PnP of batch bc - pyr_wait is done.
static int queue_batch_waits(odo_ctx* c, uint64_t bc) {
    int e;
    const int s = (int)((c->seq_set + (int)(bc - c->batch_counter) + 1) % NSETS);  // the set batch bc extracts into
    if (c->pdone_rec[s] && (e = wait_pnp_done(c, c->stream, s))) return e;
    if (c->sched == 5 && c->pyr_wait > 0 && bc >= (uint64_t)c->pyr_wait) {
        const int sb = c->batch_set[(bc - (uint64_t)c->pyr_wait) & 7];
        if (!(ODO_WAIT_DEDUP && sb == s && c->pdone_rec[s]) && (e = wait_pnp_done(c, c->stream, sb))) return e;
    }
    return ODO_OK;
}

// Stage-timing marks (odo_last_timings) are recorded only when enabled with
// odo_set_timing: timing events serialise the queue they sit on, which costs
// tens of microseconds per mark once several streams are busy.
static inline void tmark(odo_ctx* c, int i, hipStream_t st) {
    if (c->timing) hipEventRecord(c->ev[i], st);
}

// Every stream runs at the default priority: measured on MI355X, giving the
// pair / PnP streams the highest priority starves the extraction stream and
// costs 17% throughput (1.63 vs 1.35 ms per 64-frame step). ODO_STREAM_PRIO=1
// restores the high priority for experiments.
static int pair_stream_priority() {
    const char* e = odo_knob("ODO_STREAM_PRIO");
    if (!(e && e[0] == '1')) return 0;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
    return greatest;
}

// ODO_EXTRACT_STREAM_PRIO=1 (tuning): the extraction stream (the step's
// critical path) at the highest stream priority
static int extract_stream_priority() {
    const char* e = odo_knob("ODO_EXTRACT_STREAM_PRIO");
    if (!(e && e[0] == '1')) return 0;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return 0;
    return greatest;
}

// Packed layout in the staging buffer: 256-byte aligned sections
struct Pack {
    size_t off = 0;
    size_t add(size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 255) & ~(size_t)255;
        return o;
    }
};
// a typed view of a section of a packed device buffer
struct DevView {
    uint8_t* p;
    template <typename T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};
static int stage_reserve(odo_ctx* c, size_t bytes) {
    if (bytes <= c->stage_cap) return ODO_OK;
    size_t cap = std::max(bytes, std::max(c->stage_cap * 2, (size_t)1 << 20));
    if (c->stage_h) (void)hipHostFree(c->stage_h);
    c->stage_h = nullptr;
    c->stage_cap = 0;
    if (hipHostMalloc((void**)&c->stage_h, cap, hipHostMallocDefault) != hipSuccess)
        return fail(ODO_ERR_DEVICE, "hipHostMalloc (staging) failed");
    c->stage_cap = cap;
    return ODO_OK;
}

static int sync_all(odo_ctx* c) {
    for (hipStream_t st : c->owned) HIPCHK(hipStreamSynchronize(st));
    c->depth_busy = false;
    return ODO_OK;
}

static void free_ctx(odo_ctx* c) {
    if (!c) return;
    free_hyp_session(c->hs);
    void* ptrs[] = {c->lv, c->cells, c->fsegs, c->rx, c->ry, c->pyr, c->blur, c->cand, c->cand_cnt, c->keys, c->knode, c->kquad,
                    c->okp, c->ocnt, c->kps, c->desc, c->kun, c->xyz, c->ur, c->nkp, c->bgr_in[0], c->depth_in[0],
                    c->bgr_in[1], c->depth_in[1],
                    c->sort_scratch, c->latch, c->masks, c->adc, c->adb, c->smap, c->acand, c->abig, c->acell,
                    c->akp, c->aband_cnt, c->ahist, c->atsel, c->ansel, c->acell_cnt, c->athresh, c->oai, c->oac,
                    c->oab, c->cpyr, c->oscr, c->ocand, c->oband_cnt, c->ohist, c->ophist,
                    c->ocell, c->oakp};
    for (void* p : ptrs)
        if (p) hipFree(p);
    for (int i = 0; i < NSETS; i++) {
        void* pp[] = {c->knn_idx[i], c->knn_dist[i], c->rscr[i], c->lm_bits[i], c->qlist[i], c->qcnt[i]};
        for (void* q : pp)
            if (q) hipFree(q);
    }
    for (auto& P : c->pb) {
        void* pp[] = {P.matches, P.n_matches, P.n_good, P.pair_valid, P.good, P.f2_src, P.best_mask, P.res, P.T12,
                      P.edges, P.pnp_mask, P.pair_phase};
        for (void* q : pp)
            if (q) hipFree(q);
    }
    for (int i = 0; i < c->nev; i++) hipEventDestroy(c->ev[i]);
    for (int i = 0; i < odo_ctx::KT_RING; i++) {
        if (c->kt0[i]) hipEventDestroy(c->kt0[i]);
        if (c->kt1[i]) hipEventDestroy(c->kt1[i]);
    }
    if (c->kt_ref) hipEventDestroy(c->kt_ref);
    for (int i = 0; i < NSETS; i++) {
        hipEvent_t* evs[] = {&c->ev_ra[i], &c->ev_rb[i], &c->ev_pa[i], &c->ev_pb[i]};
        for (hipEvent_t* e : evs)
            if (*e) hipEventDestroy(*e);
        if (c->ev_xdone[i]) hipEventDestroy(c->ev_xdone[i]);
        if (c->ev_raw[i]) hipEventDestroy(c->ev_raw[i]);
        if (c->ev_pyr[i]) hipEventDestroy(c->ev_pyr[i]);
        if (c->ev_blur[i]) hipEventDestroy(c->ev_blur[i]);
        if (c->ev_geo[i]) hipEventDestroy(c->ev_geo[i]);
    }
    for (int i = 0; i < 2; i++) {
        if (c->ev_in_copied[i]) hipEventDestroy(c->ev_in_copied[i]);
        if (c->ev_in_free[i]) hipEventDestroy(c->ev_in_free[i]);
    }
    if (c->ev_knn) hipEventDestroy(c->ev_knn);
    if (c->ev_latch) hipEventDestroy(c->ev_latch);
    if (c->ev_depth_done) hipEventDestroy(c->ev_depth_done);
    if (c->stage_h) (void)hipHostFree(c->stage_h);
    if (c->hyp_stage_h) (void)hipHostFree(c->hyp_stage_h);
    if (c->hyp_up) hipEventDestroy(c->hyp_up);
    for (hipStream_t st : c->owned) hipStreamDestroy(st);
    if (c->h_open) (void)hipHostFree(c->h_open);
    if (c->latch_set_h) (void)hipHostFree(c->latch_set_h);
    delete c;
}

// ADAPTIVE with the cv::ORB inner detector: per grid cell the 8 levels of
// cv::ORB's pyramid of the cell sub-image (getScale sizes, orb.cpp), their
// candidate bands (rows [15, h-15) in OA_BH-row bands; strict 3x3 maxima are
// never 8-adjacent: <= ceil(r/2)ceil(c/2) survivors); the frame
// pyramid (pyr / blur, built by build_geometry) must have cv::ORB's level
// sizes, since cv::ORB::compute samples it.
static int build_adaptive_orb_geometry(odo_ctx* c) {
    const odo_adaptive_params& P = c->cfg.adaptive;
    float scale[OA_NLEV];
    int quota[OA_NLEV];
    {
        const double sf = (double)1.2f;
        const float factor = (float)(1.0 / sf);
        float nd = 10000 * (1 - factor) / (1 - (float)pow((double)factor, (double)OA_NLEV));
        int sum = 0;
        for (int l = 0; l < OA_NLEV; l++) {
            scale[l] = (float)pow(sf, (double)l);
            c->osc.s[l] = scale[l];
            if (l < OA_NLEV - 1) {
                quota[l] = cvRoundH(nd);
                sum += quota[l];
                nd *= factor;
            } else
                quota[l] = std::max(10000 - sum, 0);
        }
    }
    // the DetectorAdjuster chain runs on sum_l min(count_l, quota_l): exact
    // decisions need every quota above gridMax (k_adaptive_orb.hip)
    for (int l = 0; l < OA_NLEV; l++)
        if (quota[l] <= P.cell_max) return fail(ODO_ERR_ARG, "ADAPTIVE ORB: a level quota <= cell_max");
    if (c->nlevels < OA_NLEV) return fail(ODO_ERR_ARG, "ADAPTIVE ORB needs orb.nlevels >= 8 (frame pyramid)");
    for (int l = 0; l < OA_NLEV; l++) {
        const float inv = 1.0f / scale[l];
        if (cvRoundH((float)c->W * inv) != c->lv_h[l].w || cvRoundH((float)c->H * inv) != c->lv_h[l].h)
            return fail(ODO_ERR_ARG, "ADAPTIVE ORB: cv::ORB level size differs from the frame pyramid's");
    }
    c->oai_h.clear();
    c->oac_h.clear();
    c->oab_h.clear();
    int off = 0, coff = 0, buf0 = 0, buf1 = 0;
    c->oa_ncap = 1;
    for (const AdCell& A : c->adc_h) {
        OaCell C{};
        C.rs = A.rs;
        C.cs = A.cs;
        C.cw = A.ce - A.cs;
        C.ch = A.re - A.rs;
        C.img0 = (int)c->oai_h.size();
        int ncap = 0;
        for (int l = 0; l < OA_NLEV; l++) {
            OaImg I{};
            const float inv = 1.0f / scale[l];
            I.w = cvRoundH((float)C.cw * inv);
            I.h = cvRoundH((float)C.ch * inv);
            if (I.w > 1024 || I.h > 1024) return fail(ODO_ERR_ARG, "ADAPTIVE ORB: cell wider than 1024");
            if (I.w < 1 || I.h < 1) return fail(ODO_ERR_ARG, "ADAPTIVE ORB: empty cell level");
            I.pitch = (I.w + 15) & ~15;
            c->oa_maxpitch = std::max(c->oa_maxpitch, I.pitch);
            I.off = off;
            off += I.pitch * I.h;
            I.quota = quota[l];
            (l & 1 ? buf1 : buf0) = std::max(l & 1 ? buf1 : buf0, I.pitch * I.h);
            const int img = (int)c->oai_h.size();
            I.band0 = (int)c->oab_h.size();
            I.cand_cap = 0;
            const int cw = I.w - 2 * OA_EDGE;
            if (cw > 0)
                for (int y0 = OA_EDGE; y0 < I.h - OA_EDGE; y0 += OA_BH) {
                    OaBand B{img, y0, std::min(y0 + OA_BH, I.h - OA_EDGE), coff};
                    const int cap = ((B.y1 - B.y0 + 1) / 2) * ((cw + 1) / 2);
                    coff += (cap + 3) & ~3;
                    I.cand_cap += cap;
                    c->oab_h.push_back(B);
                }
            I.band1 = (int)c->oab_h.size();
            ncap += I.cand_cap;
            c->oai_h.push_back(I);
        }
        c->oa_ncap = std::max(c->oa_ncap, ncap);
        c->oac_h.push_back(C);
    }
    c->cp_stride = (size_t)off + 64;
    c->ocand_stride = (size_t)std::max(coff, 4);
    c->oa_buf0 = buf0;
    c->oa_buf1 = buf1;
    c->oscr_stride = (oa_select_scratch_bytes(c->oa_ncap) + 255) & ~(size_t)255;
    if (oa_scand_lds_bytes(c->oa_maxpitch) > 160 * 1024) return fail(ODO_ERR_ARG, "ADAPTIVE ORB: cell too wide for the S band");
    if (oa_assemble_lds_bytes(c->ad_ncells, c->ad_mpc) > 160 * 1024)
        return fail(ODO_ERR_ARG, "ADAPTIVE ORB grid keeps too many keypoints for one workgroup");
    if (c->ad_ncells > 15) return fail(ODO_ERR_ARG, "ADAPTIVE ORB: more than 15 grid cells");
    int e;
    if ((e = dalloc(&c->oai, c->oai_h.size()))) return e;
    if ((e = dalloc(&c->oac, c->oac_h.size()))) return e;
    if ((e = dalloc(&c->oab, std::max<size_t>(c->oab_h.size(), 1)))) return e;
    HIPCHK(hipMemcpy(c->oai, c->oai_h.data(), c->oai_h.size() * sizeof(OaImg), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->oac, c->oac_h.data(), c->oac_h.size() * sizeof(OaCell), hipMemcpyHostToDevice));
    if (!c->oab_h.empty())
        HIPCHK(hipMemcpy(c->oab, c->oab_h.data(), c->oab_h.size() * sizeof(OaBand), hipMemcpyHostToDevice));
    return ODO_OK;
}

// ADAPTIVE grid (videogridadaptedfeaturedetector.cpp:62-71): cell ROIs,
// FAST detection regions (ROI minus 3 px) and AD_BH-row bands with survivor
// capacities (strict 3x3 maxima are never 8-adjacent: <= ceil(r/2)ceil(c/2)).
static int build_adaptive_geometry(odo_ctx* c) {
    const odo_adaptive_params& P = c->cfg.adaptive;
    const int W = c->W, H = c->H, R = P.grid_rows, C = P.grid_cols, E = P.edge_threshold;
    if (R <= 0 || C <= 0 || R * C > 64 || E < 0 || P.escape_iters < 1 || P.max_total_keypoints < R * C ||
        !(P.min_thresh <= P.max_thresh))
        return fail(ODO_ERR_ARG, "invalid adaptive params");
    c->ad_ncells = R * C;
    c->ad_mpc = P.max_total_keypoints / (R * C);
    c->adc_h.clear();
    c->adb_h.clear();
    int off = 0, maxcap = 0;
    for (int i = 0; i < R; i++)
        for (int j = 0; j < C; j++) {
            AdCell A{};
            A.rs = std::max((i * H) / R - E, 0);
            A.re = std::min(H, ((i + 1) * H) / R + E);
            A.cs = std::max((j * W) / C - E, 0);
            A.ce = std::min(W, ((j + 1) * W) / C + E);
            A.r0 = A.rs + 3;
            A.r1 = std::max(A.r0, A.re - 3);
            A.c0 = A.cs + 3;
            A.c1 = std::max(A.c0, A.ce - 3);
            if (A.c1 - A.c0 > AD_MAXW) return fail(ODO_ERR_ARG, "adaptive cell wider than AD_MAXW");
            A.band0 = (int)c->adb_h.size();
            A.cand_cap = 0;
            const int cw2 = (A.c1 - A.c0 + 1) / 2;
            for (int y0 = A.r0; y0 < A.r1; y0 += AD_BH) {
                AdBand B{(int)c->adc_h.size(), y0, std::min(y0 + AD_BH, A.r1), off};
                const int cap = ((B.y1 - B.y0 + 1) / 2) * cw2;
                off += (cap + 3) & ~3;
                A.cand_cap += cap;
                c->adb_h.push_back(B);
            }
            A.band1 = (int)c->adb_h.size();
            maxcap = std::max(maxcap, A.cand_cap);
            c->adc_h.push_back(A);
        }
    c->ad_nbands = (int)c->adb_h.size();
    c->acand_stride = (size_t)std::max(off, 4);
    c->abig_stride = (size_t)3 * std::max(maxcap, 1);
    const int need = c->ad_ncells * c->ad_mpc;
    if (adapt_assemble_lds_bytes(c->ad_ncells, c->ad_mpc) > 160 * 1024)
        return fail(ODO_ERR_ARG, "adaptive grid keeps too many keypoints for one workgroup");
    c->kp_cap = std::max(c->kp_cap, (need + 63) & ~63);
    if (c->adaptive_orb) {
        int e;
        if ((e = build_adaptive_orb_geometry(c))) return e;
    }
    // ORB's rBRIEF at the FAST keypoints' angle -1 (orb.cpp computeOrbDescriptors)
    const float ang = -1.f * (float)(M_PI / 180.f);
    c->a_cos = (float)cos((double)ang);
    c->a_sin = (float)sin((double)ang);
    int e;
    if ((e = dalloc(&c->adc, c->adc_h.size()))) return e;
    if ((e = dalloc(&c->adb, std::max<size_t>(c->adb_h.size(), 1)))) return e;
    HIPCHK(hipMemcpy(c->adc, c->adc_h.data(), c->adc_h.size() * sizeof(AdCell), hipMemcpyHostToDevice));
    if (!c->adb_h.empty())
        HIPCHK(hipMemcpy(c->adb, c->adb_h.data(), c->adb_h.size() * sizeof(AdBand), hipMemcpyHostToDevice));
    return ODO_OK;
}

static int reset_adaptive(odo_ctx* c) {
    if (!c->adaptive) return ODO_OK;
    std::vector<double> t(c->ad_ncells, c->cfg.adaptive.init_thresh);
    HIPCHK(hipMemcpy(c->athresh, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
    return ODO_OK;
}

static int build_geometry(odo_ctx* c) {
    const odo_orb_params& p = c->cfg.orb;
    const int W = c->W, H = c->H;
    c->nlevels = p.nlevels;
    // ORBextractor tables (orbextractor.cpp:353-381); scaleFactor member is double
    std::vector<float> scale(p.nlevels), inv(p.nlevels);
    scale[0] = 1.0f;
    for (int i = 1; i < p.nlevels; i++) scale[i] = (float)((double)scale[i - 1] * (double)p.scale_factor);
    for (int i = 0; i < p.nlevels; i++) inv[i] = 1.0f / scale[i];
    std::vector<int> quota(p.nlevels);
    const double sf = (double)p.scale_factor;
    float factor = (float)(1.0f / sf);
    float nDesired = p.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; l++) {
        quota[l] = cvRoundH(nDesired);
        sum += quota[l];
        nDesired *= factor;
    }
    quota[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);

    c->lv_h.resize(p.nlevels);
    int off = 0, maxq = 0, max_nini = 1;
    size_t key_off = 0;
    c->cells_h.clear();
    c->fsegs_h.clear();
    int max_tiles = 0;
    for (int l = 0; l < p.nlevels; l++) {
        LevelDesc& L = c->lv_h[l];
        L.w = cvRoundH((float)W * inv[l]);
        L.h = cvRoundH((float)H * inv[l]);
        L.pitch = (L.w + 15) & ~15;
        L.off = off;
        L.scale = scale[l];
        L.quota = quota[l];
        off += L.pitch * L.h;
        maxq = std::max(maxq, quota[l]);
        if (L.w < 40 || L.h < 40) return fail(ODO_ERR_ARG, "pyramid level too small (< 40 px)");
        // FAST cells (orbextractor.cpp:669-703)
        const float Wc = 30;
        const int minBorderX = 16, minBorderY = 16;
        const int maxBorderX = L.w - 16, maxBorderY = L.h - 16;
        const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
        const int wCell = (int)ceil(width / nCols), hCell = (int)ceil(height / nRows);
        L.cell_begin = (int)c->cells_h.size();
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                CellDesc C;
                C.level = (int16_t)l;
                C.y0 = (int16_t)(int)iniY;
                C.x0 = (int16_t)(int)iniX;
                C.rows = (int16_t)((int)maxY - (int)iniY);
                C.cols = (int16_t)((int)maxX - (int)iniX);
                C.offx = (int16_t)(j * wCell);
                C.offy = (int16_t)(i * hCell);
                C.pad = 0;
                if (C.rows > FAST_ROI_MAX || C.cols > FAST_ROI_MAX) return fail(ODO_ERR_ARG, "FAST cell exceeds ROI max");
                c->cells_h.push_back(C);
                c->fast_roi = std::max(c->fast_roi, (int)std::max(C.rows, C.cols));
                c->cell_cap = std::max(c->cell_cap, ((C.rows - 6 + 1) / 2) * ((C.cols - 6 + 1) / 2) + 1);
            }
        }
        L.cell_end = (int)c->cells_h.size();
        // FAST segments (k_fast_seg): each cell row's cells in runs of at most
        // FS_SEGC whose ROI union (plus up to 15 bytes of alignment) fits the
        // FS_RS-byte LDS row, split evenly; the segment's ROI union is
        // cells_h[ci0 .. ci0 + ncell) (pushed above in row-major order)
        {
            const int nct = L.cell_end - L.cell_begin;
            int ncj = 0;  // cells per row (the skipped columns are the last ones)
            for (int j = 0; j < nCols; j++)
                if ((float)(minBorderX + j * wCell) < (float)(maxBorderX - 6)) ncj++;
            if (ncj > 0 && nct % ncj == 0) {
                const int kmax = std::min(FS_SEGC, (FS_RS - 15 - 6) / wCell);
                if (kmax < 1) return fail(ODO_ERR_ARG, "FAST cell wider than a segment row");
                const int nrow = nct / ncj, nseg = (ncj + kmax - 1) / kmax;
                for (int ir = 0; ir < nrow; ir++)
                    for (int sg = 0; sg < nseg; sg++) {
                        const int ja = ncj * sg / nseg, jb = ncj * (sg + 1) / nseg;
                        const CellDesc& A = c->cells_h[L.cell_begin + ir * ncj + ja];
                        const CellDesc& B = c->cells_h[L.cell_begin + ir * ncj + jb - 1];
                        FastSeg G{};
                        G.level = l;
                        G.ci0 = L.cell_begin + ir * ncj + ja;
                        G.y0 = A.y0;
                        G.rows = A.rows;
                        G.x0 = A.x0;
                        G.cols = (int16_t)(B.x0 + B.cols - A.x0);
                        G.ncell = (int16_t)(jb - ja);
                        G.wcell = (int16_t)wCell;
                        G.bw = (int16_t)((G.cols + 31) >> 5);
                        if ((A.x0 & 15) + G.cols > FS_RS || G.ncell > FS_NCM || G.rows > 70 || (int)G.rows * FS_RS > 65536)
                            return fail(ODO_ERR_ARG, "FAST segment too large");
                        c->fsegs_h.push_back(G);
                    }
            } else if (nct > 0) {
                return fail(ODO_ERR_STATE, "FAST cells not a full grid");
            }
        }
        L.key_off = (int)key_off;
        const int nIni = (int)roundf((float)(maxBorderX - minBorderX) / (float)(maxBorderY - minBorderY));
        max_nini = std::max(max_nini, nIni);
        const int tiles = ((L.w + 63) / 64) * ((L.h + 15) / 16);
        max_tiles = std::max(max_tiles, tiles);
    }
    c->ncells = (int)c->cells_h.size();
    c->cell_cap = (c->cell_cap + 3) & ~3;
    for (int l = 0; l < p.nlevels; l++) {
        LevelDesc& L = c->lv_h[l];
        L.key_off = 0;
    }
    size_t koff = 0;
    for (int l = 0; l < p.nlevels; l++) {
        c->lv_h[l].key_off = (int)koff;
        koff += (size_t)(c->lv_h[l].cell_end - c->lv_h[l].cell_begin) * c->cell_cap;
    }
    c->keys_per_frame = koff;
    c->pyr_size = (size_t)off + 64;  // tail: 16-byte staging loads may run past the last row
    c->max_blur_tiles = max_tiles;
    c->okp_stride = maxq + 8;
    int nc = 64;
    while (nc < std::max(maxq + 8, 4 * max_nini + 8)) nc <<= 1;
    c->node_cap = nc;
    if (octree_lds_bytes(nc) > 160 * 1024) return fail(ODO_ERR_ARG, "octree node capacity exceeds LDS");
    c->kp_cap = ((p.nfeatures + 4 * p.nlevels + 8) + 63) & ~63;
    if (c->kp_cap > 8192) return fail(ODO_ERR_ARG, "nfeatures too large (kp cap 8192)");
    if (c->adaptive) {
        int e;
        if ((e = build_adaptive_geometry(c))) return e;
        // the ADAPTIVE keypoint capacity (cells x per-cell maximum) may exceed
        // the cap checked above: the LDS landmark bit sets of k_vo_lm /
        // k_pair_match and the 13-bit train index of the kNN-2 keys hold 8192
        if (c->kp_cap > 8192) return fail(ODO_ERR_ARG, "ADAPTIVE max_total_keypoints too large (kp cap 8192)");
    }
    c->match_cap = c->kp_cap;
    c->mask_words = (c->match_cap + 31) / 32;
    // resize tables (cv::resize generic INTER_LINEAR, App. A.2)
    std::vector<ResizeX> rx;
    std::vector<ResizeY> ry;
    c->rx_off.assign(p.nlevels, 0);
    c->ry_off.assign(p.nlevels, 0);
    c->rz_rows.assign(p.nlevels, 0);
    for (int l = 1; l < p.nlevels; l++) {
        const LevelDesc& S = c->lv_h[l - 1];
        const LevelDesc& D = c->lv_h[l];
        const double inv_sx = (double)D.w / S.w, inv_sy = (double)D.h / S.h;
        const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
        c->rx_off[l] = (int)rx.size();
        std::vector<int> xofs(D.w);
        std::vector<int> a0(D.w), a1(D.w);
        int xmax = D.w;
        for (int dx = 0; dx < D.w; dx++) {
            float fx = (float)((dx + 0.5) * scale_x - 0.5);
            int sx = cvFloorH(fx);
            fx -= sx;
            if (sx < 0) {
                fx = 0;
                sx = 0;
            }
            if (sx + 1 >= S.w) {
                xmax = std::min(xmax, dx);
                if (sx >= S.w - 1) {
                    fx = 0;
                    sx = S.w - 1;
                }
            }
            xofs[dx] = sx;
            a0[dx] = satShort((1.f - fx) * 2048);
            a1[dx] = satShort(fx * 2048);
        }
        for (int dx = 0; dx < D.w; dx++) {
            ResizeX X;
            X.sx0 = xofs[dx];
            if (dx < xmax) {
                X.sx1 = xofs[dx] + 1;
                X.a0 = a0[dx];
                X.a1 = a1[dx];
            } else {
                X.sx1 = xofs[dx];
                X.a0 = 2048;
                X.a1 = 0;
            }
            rx.push_back(X);
        }
        c->ry_off[l] = (int)ry.size();
        for (int dy = 0; dy < D.h; dy++) {
            float fy = (float)((dy + 0.5) * scale_y - 0.5);
            int sy = cvFloorH(fy);
            fy -= sy;
            ResizeY Y;
            Y.b0 = satShort((1.f - fy) * 2048);
            Y.b1 = satShort(fy * 2048);
            Y.sy0 = std::min(std::max(sy, 0), S.h - 1);
            Y.sy1 = std::min(std::max(sy + 1, 0), S.h - 1);
            ry.push_back(Y);
        }
        // source rows one band of RZ_RB output rows stages in LDS
        int mr = 1;
        for (int y0 = 0; y0 < D.h; y0 += RZ_RB) {
            const int y1 = std::min(y0 + RZ_RB, D.h) - 1;
            mr = std::max(mr, ry[c->ry_off[l] + y1].sy1 - ry[c->ry_off[l] + y0].sy0 + 1);
        }
        c->rz_rows[l] = mr;
        if (resize_lds_bytes(S.pitch, D.w, mr) > 64 * 1024) return fail(ODO_ERR_ARG, "image too wide for the resize band");
    }
    c->pform = c->cfg.forms.pyramid;
    if (const char* e = odo_knob("ODO_PYRAMID_FORM")) c->pform = atoi(e);  // tuning build: A/B without a config change
    c->pyr_fusable = pyramid_fusable(c->lv_h.data(), rx.data(), c->rx_off.data(), p.nlevels);
    c->blur_fusable = c->pyr_fusable && pyramid_blur_fusable(c->lv_h.data(), p.nlevels);
    if (p.nlevels <= 16) {
    }
    int e;
    if ((e = dalloc(&c->lv, c->lv_h.size()))) return e;
    if ((e = dalloc(&c->cells, c->cells_h.size()))) return e;
    if ((e = dalloc(&c->rx, rx.size()))) return e;
    if ((e = dalloc(&c->ry, ry.size()))) return e;
    HIPCHK(hipMemcpy(c->lv, c->lv_h.data(), c->lv_h.size() * sizeof(LevelDesc), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->cells, c->cells_h.data(), c->cells_h.size() * sizeof(CellDesc), hipMemcpyHostToDevice));
    if (!fast_lds_plan(c->fsegs_h.data(), (int)c->fsegs_h.size(), c->fs_lds))
        return fail(ODO_ERR_ARG, "FAST segments exceed LDS");
    if ((e = dalloc(&c->fsegs, std::max<size_t>(c->fsegs_h.size(), 1)))) return e;
    if (!c->fsegs_h.empty())
        HIPCHK(hipMemcpy(c->fsegs, c->fsegs_h.data(), c->fsegs_h.size() * sizeof(FastSeg), hipMemcpyHostToDevice));
    if (!rx.empty()) HIPCHK(hipMemcpy(c->rx, rx.data(), rx.size() * sizeof(ResizeX), hipMemcpyHostToDevice));
    if (!ry.empty()) HIPCHK(hipMemcpy(c->ry, ry.data(), ry.size() * sizeof(ResizeY), hipMemcpyHostToDevice));
    c->ry_h = ry;
    return ODO_OK;
}

static int alloc_buffers(odo_ctx* c) {
    const size_t S = NSETS * (size_t)c->slots, B = (size_t)c->maxb;
    int e;
    if ((e = dalloc(&c->pyr, S * c->pyr_size))) return e;
    if ((e = dalloc(&c->blur, S * c->pyr_size))) return e;
    if ((e = dalloc(&c->cand, S * c->ncells * c->cell_cap))) return e;
    if ((e = dalloc(&c->cand_cnt, S * c->ncells))) return e;
    if ((e = dalloc(&c->keys, S * c->keys_per_frame))) return e;
    if ((e = dalloc(&c->knode, S * c->keys_per_frame))) return e;
    if ((e = dalloc(&c->kquad, S * c->keys_per_frame))) return e;
    if ((e = dalloc(&c->okp, S * c->nlevels * c->okp_stride))) return e;
    if ((e = dalloc(&c->ocnt, S * c->nlevels))) return e;
    if ((e = dalloc(&c->kps, S * c->kp_cap))) return e;
    if ((e = dalloc(&c->desc, S * c->kp_cap * 32))) return e;
    if ((e = dalloc(&c->kun, S * c->kp_cap * 2))) return e;
    if ((e = dalloc(&c->xyz, S * c->kp_cap * 3))) return e;
    if ((e = dalloc(&c->ur, S * c->kp_cap))) return e;
    if ((e = dalloc(&c->nkp, S))) return e;
    for (int i = 0; i < 2; i++) {
        if ((e = dalloc(&c->bgr_in[i], B * c->W * c->H * 3))) return e;
        if ((e = dalloc(&c->depth_in[i], B * c->W * c->H))) return e;
    }
    c->lm_words = (c->kp_cap + 31) / 32;
    // kernel forms (odo_config.forms; all bit-identical)
    if (c->cfg.forms.knn_split > 0) c->knn_split = std::min(8, c->cfg.forms.knn_split);
    c->knn_mx = c->cfg.forms.knn == ODO_KNN_FORM_VALU ? KNN_FMT_VALU : KNN_FMT_F4;
    if (const char* ks = odo_knob("ODO_KNN_SPLIT")) c->knn_split = std::min(8, std::max(1, atoi(ks)));
    if (const char* km = odo_knob("ODO_KNN_MFMA")) c->knn_mx = std::min(2, std::max(0, atoi(km)));
    if (c->knn_mx) c->knn_split = 1;  // one top-2 slot per query
    for (int i = 0; i < NSETS; i++) {
        if ((e = dalloc(&c->knn_idx[i], (size_t)c->knn_split * B * c->kp_cap))) return e;
        if ((e = dalloc(&c->knn_dist[i], (size_t)c->knn_split * B * c->kp_cap))) return e;
        if ((e = dalloc(&c->lm_bits[i], B * c->lm_words))) return e;
        if ((e = dalloc(&c->qlist[i], B * c->kp_cap))) return e;
        if ((e = dalloc(&c->qcnt[i], B))) return e;
    }
    for (auto& P : c->pb) {
        if ((e = dalloc(&P.matches, B * c->match_cap))) return e;
        if ((e = dalloc(&P.n_matches, B))) return e;
        if ((e = dalloc(&P.n_good, B))) return e;
        if ((e = dalloc(&P.pair_valid, B))) return e;
        if ((e = dalloc((uint64_t**)&P.good, B * c->match_cap))) return e;
        if ((e = dalloc(&P.f2_src, B * c->kp_cap))) return e;
        if ((e = dalloc(&P.best_mask, B * c->mask_words))) return e;
        if ((e = dalloc(&P.res, B))) return e;
        if ((e = dalloc(&P.T12, B * 16))) return e;
        if ((e = dalloc((uint8_t**)&P.edges, B * c->kp_cap * pnp_edge_bytes()))) return e;
        if ((e = dalloc(&P.pnp_mask, B * c->kp_cap))) return e;
        if ((e = dalloc(&P.pair_phase, B))) return e;
    }
    int pw = 1;
    while (pw < c->kp_cap) pw <<= 1;
    if ((e = dalloc(&c->sort_scratch, B * std::max(pw, c->kp_cap)))) return e;
    if ((e = dalloc(&c->latch, 1))) return e;
    for (int i = 0; i < NSETS; i++)
        if ((e = dalloc((uint8_t**)&c->rscr[i], ransac_scratch_bytes((int)B, c->match_cap, c->mask_words, c->rcfg))))
            return e;

    if (c->adaptive) {
        const size_t nc = (size_t)c->ad_ncells;
        if ((e = dalloc(&c->atsel, B * nc))) return e;
        if ((e = dalloc(&c->ansel, B * nc))) return e;
        if ((e = dalloc(&c->acell_cnt, B * nc))) return e;
        if ((e = dalloc(&c->athresh, nc))) return e;
        if (!c->adaptive_orb) {
            c->smap_stride = (size_t)c->lv_h[0].pitch * c->H;
            if ((e = dalloc(&c->smap, B * c->smap_stride))) return e;
            if ((e = dalloc(&c->acand, B * c->acand_stride))) return e;
            if ((e = dalloc(&c->aband_cnt, B * std::max(c->ad_nbands, 1)))) return e;
            if ((e = dalloc(&c->ahist, B * nc * 256))) return e;
            if ((e = dalloc(&c->abig, B * nc * c->abig_stride))) return e;
            if ((e = dalloc(&c->acell, B * nc * c->ad_mpc))) return e;
            if ((e = dalloc(&c->akp, B * c->kp_cap))) return e;
        } else {
            const size_t ni = c->oai_h.size();
            if ((e = dalloc(&c->cpyr, B * c->cp_stride))) return e;
            if ((e = dalloc(&c->ocand, B * c->ocand_stride))) return e;
            if ((e = dalloc(&c->oband_cnt, B * std::max<size_t>(c->oab_h.size(), 1)))) return e;
            if ((e = dalloc(&c->ohist, B * ni * 256))) return e;
            if ((e = dalloc(&c->ophist, B * nc * 256))) return e;
            if ((e = dalloc(&c->oscr, B * nc * c->oscr_stride))) return e;
            if ((e = dalloc(&c->ocell, B * nc * c->ad_mpc))) return e;
            if ((e = dalloc(&c->oakp, B * c->kp_cap))) return e;
        }
        if ((e = reset_adaptive(c))) return e;
    }
    HIPCHK(hipHostMalloc((void**)&c->h_open, NSETS * sizeof(int), hipHostMallocDefault));
    for (int i = 0; i < NSETS; i++) c->h_open[i] = -1;  // unknown: the first RANSAC launch runs both forms
    HIPCHK(hipHostMalloc((void**)&c->latch_set_h, sizeof(int), hipHostMallocCoherent));
    *c->latch_set_h = 0;
    HIPCHK(hipMemset(c->nkp, 0, S * sizeof(int)));
    const double nan = std::nan("");
    HIPCHK(hipMemcpy(c->latch, &nan, sizeof(double), hipMemcpyHostToDevice));
    return ODO_OK;
}

extern "C" {

const char* odo_last_error(void) { return g_err.c_str(); }

int odo_abi_version(void) { return ODO_ABI_VERSION; }

void odo_default_config(odo_config* cfg, int width, int height, int max_batch) {
    memset(cfg, 0, sizeof(*cfg));
    cfg->struct_size = (uint32_t)sizeof(odo_config);
    cfg->width = width;
    cfg->height = height;
    cfg->max_batch = max_batch;
    cfg->orb = odo_orb_params{1000, 1.2f, 8, 20, 7};
    cfg->calib = odo_calib{517.3f, 516.5f, 318.6f, 255.3f, 0.262383f, -0.953104f, -0.005358f, 0.002628f, 1.163314f,
                           1.0f / 5000.0f, 40.0f, 40.0f};
    cfg->nn_ratio = 0.9f;
    cfg->ransac = odo_ransac_params{200, 20, 3.0f, 4, 1};
    cfg->seed = 0x5EED0000u;
    cfg->detector = ODO_DETECTOR_ORB_SLAM2;
    // Extractor::CreateAdaptiveDetector (extractor.cpp:55-77): minFeatures 600,
    // maxFeatures = 600 * 1.7 = 1020, 3x3 grid, gridMin = round(600/9.f) = 67,
    // gridMax = round(1020/9.f) = 113, 5 iterations, edge 31; FAST adjuster
    // (20, 2, 10000, 1.3, 0.7); Extract's retainBest(nFeatures = 1000)
    cfg->adaptive = odo_adaptive_params{3, 3, 31, 1020, 67, 113, 5, 20.0, 2.0, 10000.0, 1.3, 0.7, 1000};
}

odo_ctx* odo_create(const odo_config* cfg, int device) {
    if (cfg && cfg->struct_size != (uint32_t)sizeof(odo_config)) {
        char msg[160];
        snprintf(msg, sizeof(msg), "odo_config.struct_size %u != %zu: the caller was built against another odo.h "
                 "(ODO_ABI_VERSION %d); fill it with odo_default_config", cfg->struct_size, sizeof(odo_config),
                 ODO_ABI_VERSION);
        fail(ODO_ERR_ARG, msg);
        return nullptr;
    }
    if (!cfg || cfg->width <= 0 || cfg->height <= 0 || cfg->max_batch <= 0 || cfg->orb.nlevels <= 0 ||
        cfg->orb.nlevels > 16) {
        fail(ODO_ERR_ARG, "invalid config");
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) {
        fail(ODO_ERR_DEVICE, "no HIP device available (the MI355X path has no CPU fallback)");
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fail(ODO_ERR_DEVICE, std::string("device is not gfx950: ") + prop.gcnArchName);
        return nullptr;
    }
    hipSetDevice(device);
    odo_ctx* c = new odo_ctx();
    c->cfg = *cfg;
    c->device = device;
    c->W = cfg->width;
    c->H = cfg->height;
    c->maxb = cfg->max_batch;
    c->slots = cfg->max_batch + 1;
    if (cfg->forms.knn != ODO_KNN_FORM_FP4 && cfg->forms.knn != ODO_KNN_FORM_VALU) {
        fail(ODO_ERR_ARG, "unknown kNN-2 kernel form");
        delete c;
        return nullptr;
    }
    if (cfg->forms.pyramid < ODO_PYRAMID_FORM_AUTO || cfg->forms.pyramid > ODO_PYRAMID_FORM_FUSED) {
        fail(ODO_ERR_ARG, "unknown pyramid kernel form");
        delete c;
        return nullptr;
    }
    if (cfg->forms.ransac_first_hyps < 0 || cfg->forms.ransac_first_hyps > 64) {
        fail(ODO_ERR_ARG, "ransac_first_hyps: 0 (default) or 1..64");
        delete c;
        return nullptr;
    }
    if (cfg->detector != ODO_DETECTOR_ORB_SLAM2 && cfg->detector != ODO_DETECTOR_ADAPTIVE_FAST &&
        cfg->detector != ODO_DETECTOR_ADAPTIVE_ORB) {
        fail(ODO_ERR_ARG, "unsupported detector");  // extractor.cpp:26-27 terminates here
        delete c;
        return nullptr;
    }
    c->adaptive = cfg->detector == ODO_DETECTOR_ADAPTIVE_FAST || cfg->detector == ODO_DETECTOR_ADAPTIVE_ORB;
    c->adaptive_orb = cfg->detector == ODO_DETECTOR_ADAPTIVE_ORB;
    // ODO_SERIAL_STREAMS=1 (profiling): every stage on one stream, no overlap,
    // so per-kernel times are free of cross-stream contention
    const char* ser = odo_knob("ODO_SERIAL_STREAMS");
    c->serial = ser && ser[0] == '1';
    if (const char* sk = odo_knob("ODO_SKIP")) c->skip = atoi(sk);
    if (const char* sc = odo_knob("ODO_SCHED")) c->sched = atoi(sc);
    // only the streams the schedule uses (each extra stream shares one of the
    // process's GPU_MAX_HW_QUEUES hardware queues with another and serialises
    // against it); the others alias
    // ODO_PAIR_CUMASK / ODO_EXTRACT_CUMASK (tuning): comma-separated 32-bit
    // hex words of a CU mask for the pair / extraction streams (spatial
    // partitioning of the CUs between the latency-bound pair stages and the
    // throughput-bound extraction)
    auto parse_mask = [](const char* e, std::vector<uint32_t>& m) {
        m.clear();
        while (e && *e) {
            char* end = nullptr;
            m.push_back((uint32_t)strtoul(e, &end, 16));
            if (end == e) break;
            e = *end == ',' ? end + 1 : end;
        }
        return !m.empty();
    };
    std::vector<uint32_t> pmask, xmask;
    const bool pm = parse_mask(odo_knob("ODO_PAIR_CUMASK"), pmask);
    const bool xm = parse_mask(odo_knob("ODO_EXTRACT_CUMASK"), xmask);
    auto mk = [&](hipStream_t* s, bool prio) {
        bool r;
        if (prio && pm)
            r = hipExtStreamCreateWithCUMask(s, (uint32_t)pmask.size(), pmask.data()) == hipSuccess;
        else if (!prio && xm)
            r = hipExtStreamCreateWithCUMask(s, (uint32_t)xmask.size(), xmask.data()) == hipSuccess;
        else if (!prio && s == &c->stream && extract_stream_priority() != 0)
            r = hipStreamCreateWithPriority(s, hipStreamNonBlocking, extract_stream_priority()) == hipSuccess;
        else
            r = prio ? hipStreamCreateWithPriority(s, hipStreamNonBlocking, pair_stream_priority()) == hipSuccess
                     : hipStreamCreateWithFlags(s, hipStreamNonBlocking) == hipSuccess;
        if (r) c->owned.push_back(*s);
        return r;
    };
    bool ok = mk(&c->stream, false);
    if (ok && c->serial) {
        c->pstream = c->pstream2 = c->side = c->pnpa = c->pnpb = c->stream;
    } else if (ok && c->sched == 5) {
        if (const char* np = odo_knob("ODO_PSTREAMS")) c->npstreams = std::min(3, std::max(1, atoi(np)));
        if (const char* kp = odo_knob("ODO_KNN_PAIR")) c->knn_pair = atoi(kp) != 0;
        if (const char* kg = odo_knob("ODO_KNN_GATE")) c->knn_gate = atoi(kg) != 0;
        if (const char* pw = odo_knob("ODO_PYR_WAIT")) c->pyr_wait = std::min(NSETS - 1, std::max(0, atoi(pw)));
        ok = mk(&c->pstream, true) && (c->npstreams < 2 || mk(&c->pstream2, true)) &&
             (c->npstreams < 3 || mk(&c->pstream3, true));
        if (c->npstreams < 2) c->pstream2 = c->pstream;
        if (c->npstreams < 3) c->pstream3 = c->pstream;
        c->side = c->pnpa = c->pnpb = c->pstream;
        const char* bs = odo_knob("ODO_BLUR_STREAM");
        if (ok && bs && atoi(bs) != 0) ok = mk(&c->bstream, false);
    } else if (ok) {
        ok = mk(&c->pstream, true) && mk(&c->pnpa, true) && (c->sched == 0 || mk(&c->side, false)) &&
             (c->sched != 1 || mk(&c->pnpb, true));
        if (c->sched == 0) c->side = c->stream;
        if (c->sched != 1) c->pnpb = c->pnpa;
        c->pstream2 = c->pstream;
    }
    // The context's events only order its streams against each other (and
    // tell the host that inputs were consumed): none needs the system-scope
    // cache writeback + invalidate a default event record performs, which on
    // this part also disturbs every kernel then running (round 5: ~10 records
    // per batch; DESIGN §4 Pipelining)
    const unsigned evf = ODO_SYNC_EVENT_FLAGS;
    for (int i = 0; i < NSETS && ok; i++)
        ok = hipEventCreateWithFlags(&c->ev_ra[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_rb[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_pa[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_pb[i], evf) == hipSuccess;
    for (int i = 0; i < NSETS && ok; i++)
        ok = hipEventCreateWithFlags(&c->ev_xdone[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_raw[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_pyr[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_blur[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_geo[i], evf) == hipSuccess;
    if (!c->bstream) c->bstream = c->stream;
    if (ok) ok = hipEventCreateWithFlags(&c->ev_latch, evf) == hipSuccess;
    if (ok) ok = hipEventCreateWithFlags(&c->ev_depth_done, evf) == hipSuccess;
    if (ok) ok = hipEventCreateWithFlags(&c->ev_knn, evf) == hipSuccess;
    // host-input uploads run on their own stream (the DMA engines), ordered
    // against the extraction stream by events only
    if (ok) ok = mk(&c->cstream, false);
    for (int i = 0; i < 2 && ok; i++)
        ok = hipEventCreateWithFlags(&c->ev_in_copied[i], evf) == hipSuccess &&
             hipEventCreateWithFlags(&c->ev_in_free[i], evf) == hipSuccess;
    if (!ok) {
        fail(ODO_ERR_DEVICE, "hipStreamCreate failed");
        free_ctx(c);
        return nullptr;
    }
    // ErrorFunction2 statics (ransac.cpp:352-359)
    const double cam_angle_x = 58.0 / 180.0 * M_PI, cam_angle_y = 45.0 / 180.0 * M_PI;
    const double rsx = 3 * tan(cam_angle_x / 640.0), rsy = 3 * tan(cam_angle_y / 480.0);
    c->rcfg = RansacCfg{cfg->ransac.iterations, cfg->ransac.min_inlier_th, cfg->ransac.max_mahalanobis,
                        cfg->ransac.sample_size, cfg->ransac.check_depth, rsx * rsx, rsy * rsy, 0,
                        cfg->forms.ransac_lanes_min_open, 0, cfg->forms.ransac_first_hyps};
    if (build_geometry(c) != ODO_OK || alloc_buffers(c) != ODO_OK) {
        free_ctx(c);
        return nullptr;
    }
    upload_extract_constants();
    upload_adaptive_constants();
    upload_adaptive_orb_constants();
    const odo_calib& k = cfg->calib;
    c->cal = FrameCalib{k.fx, k.fy, k.cx, k.cy, k.k1, k.k2, k.p1, k.p2, k.k3, k.depth_factor, k.mbf,
                        1.0f / k.fx, 1.0f / k.fy};
    c->nev = 11;
    for (int i = 0; i < c->nev; i++) hipEventCreate(&c->ev[i]);
    return c;
}

void odo_destroy(odo_ctx* ctx) { free_ctx(ctx); }

void* odo_stream(odo_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int odo_reset(odo_ctx* c) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    int e;
    if ((e = sync_all(c))) return e;
    c->has_prev = false;
    c->pair_counter = 0;
    const double nan = std::nan("");
    HIPCHK(hipMemcpy(c->latch, &nan, sizeof(double), hipMemcpyHostToDevice));
    if (c->latch_set_h) *c->latch_set_h = 0;
    return reset_adaptive(c);
}

int odo_set_latch(odo_ctx* c, double cov) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    int e;
    if ((e = sync_all(c))) return e;
    HIPCHK(hipMemcpy(c->latch, &cov, sizeof(double), hipMemcpyHostToDevice));
    if (c->latch_set_h) *c->latch_set_h = std::isnan(cov) ? 0 : 1;
    return ODO_OK;
}

double odo_get_latch(odo_ctx* c) {
    double v = std::nan("");
    if (!c || sync_all(c)) return v;
    hipMemcpy(&v, c->latch, sizeof(double), hipMemcpyDeviceToHost);
    return v;
}

int odo_set_timing(odo_ctx* c, int mode) {
    if (!c || mode < 0 || mode > 2) return fail(ODO_ERR_ARG, "bad timing mode");
    int e;
    if ((e = sync_all(c))) return e;
    c->timing = mode == 1;
    c->ktiming = mode == 2;
    if (c->ktiming) {
        // timing only: no system-scope fence at the records (see ODO_EVFENCE)
        const unsigned tf = ODO_EVFENCE == 1 ? hipEventDisableSystemFence : 0u;
        if (!c->kt0[0])
            for (int i = 0; i < odo_ctx::KT_RING; i++)
                if (hipEventCreateWithFlags(&c->kt0[i], tf) != hipSuccess || hipEventCreateWithFlags(&c->kt1[i], tf) != hipSuccess)
                    return fail(ODO_ERR_DEVICE, "hipEventCreate failed");
        c->kt_next = c->kt_pending = 0;
        c->kt_sum_ms = 0;
        c->kt_count = 0;
        if (!c->kt_ref && hipEventCreateWithFlags(&c->kt_ref, tf) != hipSuccess)
            return fail(ODO_ERR_DEVICE, "hipEventCreate failed");
        HIPCHK(hipEventRecord(c->kt_ref, c->stream));  // every stream is idle (sync_all above)
        c->kt_marks.clear();
    }
    return ODO_OK;
}

// fold the elapsed time of ring slot i into the running sum (waits for it)
static int kt_collect(odo_ctx* c, int i) {
    HIPCHK(hipEventSynchronize(c->kt1[i]));
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, c->kt0[i], c->kt1[i]));
    c->kt_sum_ms += t;
    c->kt_count++;
    float m = 0;
    HIPCHK(hipEventElapsedTime(&m, c->kt_ref, c->kt0[i]));
    c->kt_marks.push_back(m);
    return ODO_OK;
}

int odo_kernel_timing(odo_ctx* c, double* avg_ms, long* launches) {
    if (!c || !avg_ms || !launches) return fail(ODO_ERR_ARG, "null arg");
    if (!c->ktiming) return fail(ODO_ERR_ARG, "kernel timing is off (odo_set_timing mode 2)");
    int e;
    if ((e = sync_all(c))) return e;
    const int n = c->kt_pending;
    for (int k = 0; k < n; k++) {
        const int i = (c->kt_next - n + k + odo_ctx::KT_RING) % odo_ctx::KT_RING;
        if ((e = kt_collect(c, i))) return e;
    }
    c->kt_pending = 0;
    *launches = c->kt_count;
    *avg_ms = c->kt_count ? c->kt_sum_ms / (double)c->kt_count : 0.0;
    return ODO_OK;
}

// The kNN-2 launch of batch b starts once b's extraction has finished (and
// its pair stream is free): the marks' differences are the pipeline's
// per-step times, read without adding any event to the extraction stream.
int odo_step_marks(odo_ctx* c, double* ms, int cap) {
    if (!c || cap < 0 || (cap > 0 && !ms)) return fail(ODO_ERR_ARG, "step_marks: bad arguments");
    double avg = 0;
    long n = 0;
    int e;
    if ((e = odo_kernel_timing(c, &avg, &n))) return e;  // collects the pending marks
    const int k = (int)c->kt_marks.size();
    for (int i = 0; i < k && i < cap; i++) ms[i] = c->kt_marks[i];
    return k;
}

int odo_synchronize(odo_ctx* c) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    return sync_all(c);
}

// gray (when d_bgr is given) and the pyramid levels of n frames
// (and, with blur given and c->blur_fused, the blurred levels in the same launch)
// Returns true when the blurred levels were written too.
constexpr int PYR_FUSED_MIN_FRAMES = 128;
static bool build_pyramid(odo_ctx* c, hipStream_t st, const uint8_t* d_bgr, uint8_t* pyr, int n, uint8_t* blur) {
    const size_t P = c->pyr_size;
    const bool fused = c->pyr_fusable && (c->pform == ODO_PYRAMID_FORM_FUSED || c->pform == ODO_PYRAMID_FORM_FUSED_NOBLUR ||
                                          (c->pform == ODO_PYRAMID_FORM_AUTO && n >= PYR_FUSED_MIN_FRAMES));
    if (fused) {
        if (c->pform == ODO_PYRAMID_FORM_FUSED_NOBLUR || !c->blur_fusable) blur = nullptr;
        static const bool gray_apart = [] {  // tuning: gray as its own launch before the fused levels
            const char* e = odo_knob("ODO_PYR_GRAY");
            return e && e[0] == '1';
        }();
        if (gray_apart && d_bgr) {
            launch_gray(st, d_bgr, pyr, c->W, c->H, c->lv_h[0].pitch, (size_t)c->W * c->H * 3, P, n);
            d_bgr = nullptr;
        }
        launch_pyramid(st, d_bgr, pyr, (size_t)c->W * c->H * 3, P, c->lv, c->rx, c->ry, c->rx_off.data(),
                       c->ry_off.data(), c->nlevels, n, blur, c->lv_h.data(),
                       c->ry_h.data());
        return blur != nullptr;
    }
    if (d_bgr) launch_gray(st, d_bgr, pyr, c->W, c->H, c->lv_h[0].pitch, (size_t)c->W * c->H * 3, P, n);
    for (int l = 1; l < c->nlevels; l++) {
        const LevelDesc& S = c->lv_h[l - 1];
        const LevelDesc& D = c->lv_h[l];
        launch_resize(st, pyr, P, S.off, S.pitch, D.off, D.pitch, D.w, D.h, RZ_RB, c->rz_rows[l],
                      c->rx + c->rx_off[l], c->ry + c->ry_off[l], n);
    }
    return false;
}

// Extractor(FAST, ORB, ADAPTIVE) for frames slot0.. of `set` (k_adaptive.hip):
// threshold-free S map -> band survivors + S histograms -> the per-cell
// threshold chain over the batch in frame order -> keepStrongest ->
// retainBest + border filter -> rBRIEF / undistort / depth.
static int run_extract_adaptive(odo_ctx* c, int set, const uint8_t* d_bgr, const uint16_t* d_depth, int n,
                                int slot0) {
    hipStream_t st = c->stream;
    const size_t P = c->pyr_size;
    const size_t slot = fbase(c, set) + slot0;
    const LevelDesc& L0 = c->lv_h[0];
    uint8_t* pyr = c->pyr + slot * P;
    const size_t nc = (size_t)c->ad_ncells;
    if (d_bgr) launch_gray(st, d_bgr, pyr, c->W, c->H, L0.pitch, (size_t)c->W * c->H * 3, P, n);
    tmark(c, 1, st);
    const bool split = c->bstream != st;  // blur beside the detector
    if (split) {
        HIPCHK(hipEventRecord(c->ev_pyr[set], st));
        HIPCHK(hipStreamWaitEvent(c->bstream, c->ev_pyr[set], 0));
        launch_blur(c->bstream, pyr, c->blur + slot * P, P, c->lv, c->lv_h.data(), 1, n);
        HIPCHK(hipEventRecord(c->ev_blur[set], c->bstream));
    }
    launch_adapt_smap(st, pyr, P, c->W, c->H, L0.pitch, c->smap, c->smap_stride, n);
    HIPCHK(hipMemsetAsync(c->ahist, 0, (size_t)n * nc * 256 * sizeof(int), st));
    if (c->ad_nbands > 0)
        launch_adapt_cand(st, c->smap, c->smap_stride, L0.pitch, c->adb, c->ad_nbands, c->adc, c->ad_ncells, c->acand,
                          c->acand_stride, c->aband_cnt, c->ahist, n);
    tmark(c, 2, st);
    launch_adapt_chain(st, c->ahist, c->ad_ncells, n, c->cfg.adaptive, c->athresh, c->atsel, c->ansel);
    launch_adapt_select(st, c->acand, c->acand_stride, c->aband_cnt, c->ad_nbands, c->adb, c->adc, c->ad_ncells,
                        c->atsel, c->ansel, c->ad_mpc, c->abig, c->abig_stride, c->acell, c->acell_cnt, n);
    launch_adapt_assemble(st, c->acell, c->acell_cnt, c->ad_ncells, c->ad_mpc, c->cfg.adaptive.retain_best, c->W,
                          c->H, c->akp, c->kp_cap, c->nkp + slot, c->kp_cap, n);
    tmark(c, 3, st);
    if (split)
        HIPCHK(hipStreamWaitEvent(st, c->ev_blur[set], 0));
    else
        launch_blur(st, pyr, c->blur + slot * P, P, c->lv, c->lv_h.data(), 1, n);
    tmark(c, 4, st);
    launch_adapt_finalize(st, c->blur + slot * P, P, L0.pitch, c->akp, c->kp_cap, c->nkp + slot, c->a_cos, c->a_sin,
                          d_depth, (size_t)c->W * c->H, c->W, c->cal, c->kps + slot * c->kp_cap,
                          c->desc + slot * c->kp_cap * 32, c->kun + slot * c->kp_cap * 2, c->xyz + slot * c->kp_cap * 3,
                          c->ur + slot * c->kp_cap, c->kp_cap, n);
    tmark(c, 5, st);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

// Extractor(ORB, ORB, ADAPTIVE) for frames slot0.. of `set`
// (k_adaptive_orb.hip): the frame pyramid + blur (cv::ORB::compute's levels)
// -> cell pyramids -> S maps -> band survivors + S histograms -> count tables
// -> the per-cell threshold chain -> per-cell select -> assemble ->
// IC angle / rBRIEF / undistort / depth.
static int run_extract_adaptive_orb(odo_ctx* c, int set, const uint8_t* d_bgr, const uint16_t* d_depth, int n,
                                    int slot0) {
    hipStream_t st = c->stream;
    const size_t P = c->pyr_size;
    const size_t slot = fbase(c, set) + slot0;
    uint8_t* pyr = c->pyr + slot * P;
    const int nc = c->ad_ncells, ni = (int)c->oai_h.size(), nb = (int)c->oab_h.size();
    build_pyramid(c, st, d_bgr, pyr, n, nullptr);
    tmark(c, 1, st);
    launch_oa_pyr(st, pyr, P, c->lv_h[0].pitch, c->oac, nc, c->oai, c->oa_buf0, c->oa_buf1, c->cpyr, c->cp_stride, n);
    HIPCHK(hipMemsetAsync(c->ohist, 0, (size_t)n * ni * 256 * sizeof(int), st));
    if (nb > 0)
        launch_oa_scand(st, c->cpyr, c->cp_stride, c->oai, ni, c->oab, nb, c->ocand, c->ocand_stride, c->oband_cnt,
                        c->ohist, c->oa_maxpitch, n);
    launch_oa_count(st, c->ohist, c->oac, c->oai, ni, nc, c->ophist, n);
    tmark(c, 2, st);
    launch_adapt_chain(st, c->ophist, nc, n, c->cfg.adaptive, c->athresh, c->atsel, c->ansel);
    launch_oa_select(st, c->ocand, c->ocand_stride, c->oband_cnt, nb, c->oab, c->oai, c->oac, nc, c->atsel, c->cpyr,
                     c->cp_stride, c->ad_mpc, c->oscr, c->oscr_stride, c->oa_ncap, c->ocell, c->acell_cnt, n);
    launch_oa_assemble(st, c->ocell, c->acell_cnt, c->oac, nc, c->ad_mpc, c->cfg.adaptive.retain_best, c->W, c->H,
                       c->osc, c->oakp, c->kp_cap, c->nkp + slot, c->kp_cap, n);
    tmark(c, 3, st);
    launch_blur(st, pyr, c->blur + slot * P, P, c->lv, c->lv_h.data(), OA_NLEV, n);
    tmark(c, 4, st);
    launch_oa_finalize(st, pyr, c->blur + slot * P, P, c->lv, c->cpyr, c->cp_stride, c->oai, c->oac, c->osc, c->oakp,
                       c->kp_cap, c->nkp + slot, d_depth, (size_t)c->W * c->H, c->W, c->cal,
                       c->kps + slot * c->kp_cap, c->desc + slot * c->kp_cap * 32, c->kun + slot * c->kp_cap * 2,
                       c->xyz + slot * c->kp_cap * 3, c->ur + slot * c->kp_cap, c->kp_cap, n);
    tmark(c, 5, st);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

static int run_extract(odo_ctx* c, int set, const uint8_t* d_bgr, const uint16_t* d_depth, int n, int slot0) {
    if (c->adaptive_orb) return run_extract_adaptive_orb(c, set, d_bgr, d_depth, n, slot0);
    if (c->adaptive) return run_extract_adaptive(c, set, d_bgr, d_depth, n, slot0);
    hipStream_t st = c->stream;
    const size_t P = c->pyr_size;
    const size_t slot = fbase(c, set) + slot0;
    uint8_t* pyr = c->pyr + (size_t)slot * P;
    const bool blur_done = build_pyramid(c, st, d_bgr, pyr, n, c->blur + (size_t)slot * P);
    tmark(c, 1, st);
    const bool split = c->bstream != st && !blur_done;  // blur beside FAST + octree
    if (split) {
        HIPCHK(hipEventRecord(c->ev_pyr[set], st));
        HIPCHK(hipStreamWaitEvent(c->bstream, c->ev_pyr[set], 0));
        launch_blur(c->bstream, pyr, c->blur + (size_t)slot * P, P, c->lv, c->lv_h.data(), c->nlevels, n);
        HIPCHK(hipEventRecord(c->ev_blur[set], c->bstream));
    }
    launch_fast(st, pyr, P, c->fsegs, (int)c->fsegs_h.size(), c->lv, c->cand + (size_t)slot * c->ncells * c->cell_cap,
                c->cand_cnt + (size_t)slot * c->ncells, c->ncells, c->cell_cap, c->cfg.orb.ini_th_fast,
                c->cfg.orb.min_th_fast, c->fs_lds, n);
    tmark(c, 2, st);
    launch_octree(st, c->cand + (size_t)slot * c->ncells * c->cell_cap, c->cand_cnt + (size_t)slot * c->ncells, c->lv,
                  c->ncells, c->cell_cap, c->nlevels, c->keys + (size_t)slot * c->keys_per_frame,
                  c->knode + (size_t)slot * c->keys_per_frame, c->kquad + (size_t)slot * c->keys_per_frame,
                  c->keys_per_frame, c->okp + (size_t)slot * c->nlevels * c->okp_stride,
                  c->ocnt + (size_t)slot * c->nlevels, c->okp_stride, c->node_cap, n);
    tmark(c, 3, st);
    if (c->early_waits) {
        // ODO_EARLY_WAIT: the next batch's frame-set and PYR_WAIT waits, queued
        // here, ahead of this batch's finalize, instead of between its end and
        // the next pyramid (their events were recorded by earlier batches)
        int e;
        if ((e = queue_batch_waits(c, c->batch_counter + 1))) return e;
        c->pre_waited = c->batch_counter + 1;
    }
    if (split)
        HIPCHK(hipStreamWaitEvent(st, c->ev_blur[set], 0));
    else if (!blur_done)
        launch_blur(st, pyr, c->blur + (size_t)slot * P, P, c->lv, c->lv_h.data(), c->nlevels, n);
    tmark(c, 4, st);
    launch_finalize(st, pyr, c->blur + (size_t)slot * P, P, c->lv, c->nlevels,
                    c->okp + (size_t)slot * c->nlevels * c->okp_stride, c->ocnt + (size_t)slot * c->nlevels,
                    c->okp_stride, d_depth, (size_t)c->W * c->H, c->W, c->cal, c->kps + (size_t)slot * c->kp_cap,
                    c->desc + (size_t)slot * c->kp_cap * 32, c->kun + (size_t)slot * c->kp_cap * 2,
                    c->xyz + (size_t)slot * c->kp_cap * 3, c->ur + (size_t)slot * c->kp_cap, c->nkp + slot, c->kp_cap,
                    n, !c->geo_pair);
    tmark(c, 5, st);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

// Extraction when level 0 (the gray image) is already in the pyramid slot.
static int run_extract_from_gray(odo_ctx* c, int set, const uint16_t* d_depth, int n, int slot) {
    return run_extract(c, set, nullptr, d_depth, n, slot);
}

// Extraction only (no pairs, no roll): frames land in the set the next
// tracked batch will use, so the tracking sequence state is untouched.
int odo_extract_batch(odo_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, int n) {
    if (!c || !d_bgr || !d_depth || n <= 0 || n > c->maxb) return fail(ODO_ERR_ARG, "bad extract args");
    int e;
    if ((e = sync_all(c))) return e;
    const int set = next_set(c);
    tmark(c, 0, c->stream);
    if ((e = run_extract(c, set, d_bgr, d_depth, n, 1))) return e;
    c->view_set = set;
    c->last_n = n;
    return ODO_OK;
}

// Pair stages of one batch on the pair stream, over frame set `set`:
// pair p is (slot p, slot p+1); pair 0 is valid only with a previous frame.
static int run_pairs(odo_ctx* c, int set, int n) {
    hipStream_t st = c->cur_p ? c->cur_p : c->pstream;
    auto& P = c->pb[set];
    const size_t KC = (size_t)c->kp_cap;
    const size_t b = fbase(c, set);
    uint8_t* desc = c->desc + b * KC * 32;
    int* nkp = c->nkp + b;
    float* xyz = c->xyz + b * KC * 3;
    tmark(c, 6, st);
    launch_pair_valid(st, P.pair_valid, n, c->has_prev ? 1 : 0);
    launch_pair_match(st, c->knn_idx[set], c->knn_dist[set], KC, xyz, nkp, c->kp_cap, 0, c->cfg.nn_ratio,
                      c->lm_bits[set], c->lm_words, c->knn_split, (size_t)c->maxb * KC, c->cfg.ransac.check_depth, P.matches, P.n_matches, P.good, P.n_good, P.f2_src,
                      c->sort_scratch, c->match_cap, n);
    // the DepthCovariance latch is taken from the first valid pair ever: with
    // two pair streams, a batch's latch kernel runs after the previous one's
    // Once the latch holds a value (k_latch's host flag) and the kernel that
    // set it has completed (ev_latch), the latch kernel is a no-op: it and its
    // two ordering packets are left out (ODO_WAIT_DEDUP)
    if (!c->latched) {
        if (c->sched == 5 && c->latch_rec) HIPCHK(hipStreamWaitEvent(st, c->ev_latch, 0));
        launch_latch(st, c->latch, P.good, P.n_good, P.n_matches, P.matches, xyz, c->kp_cap, 0, n, c->match_cap,
                     c->cfg.ransac.min_inlier_th, c->cfg.ransac.sample_size, c->cfg.ransac.iterations, P.pair_valid,
                     c->latch_set_h);
        if (c->sched == 5) {
            HIPCHK(hipEventRecord(c->ev_latch, st));
            c->latch_rec = true;
        }
    }
    tmark(c, 7, st);
    if (c->sched != 1) {
        // both RANSAC launches on the pair stream, then one PnP launch for the
        // whole batch on its own stream (the pair stream moves on to the next
        // batch while it runs)
        if (!(c->skip & 16))
        launch_ransac(st, P.good, P.n_good, P.n_matches, P.matches, xyz, c->kp_cap, 0, c->match_cap, c->rcfg,
                      c->latch, P.pair_valid, 20, nullptr, c->rscr[set], P.best_mask, c->mask_words, P.res, P.T12, n,
                      0, P.pair_phase, c->h_open + set);
        tmark(c, 8, st);
        // schedule 5: PnP follows RANSAC on the batch's own pair stream, and
        // nothing waits on ev_rb (the side stream of schedules 0-3 does): no
        // marker packet between the RANSAC and PnP launches (ODO_WAIT_DEDUP)
        if (!(ODO_WAIT_DEDUP && c->sched == 5)) HIPCHK(hipEventRecord(c->ev_rb[set], st));
        hipStream_t ps = c->sched == 5 ? st : c->pnpa;
        if (ps != st) HIPCHK(hipStreamWaitEvent(ps, c->ev_rb[set], 0));
        if (!(c->skip & 1))
            launch_pnp(ps, P.f2_src, xyz, c->kun + b * KC * 2, c->ur + b * KC, nkp, c->kp_cap, 0, c->cal, P.T12,
                       P.pair_valid, P.n_matches, 20, P.edges, P.res, P.pnp_mask, n);
        tmark(c, 9, ps);
        // schedule 5 waits on ev_pb alone (wait_pnp_done), and an async batch
        // records it again after its result copy, before anything waits on it
        if (!(ODO_WAIT_DEDUP && c->sched == 5)) HIPCHK(hipEventRecord(c->ev_pa[set], ps));
        if (!(ODO_WAIT_DEDUP && c->sched == 5 && c->defer_pdone)) HIPCHK(hipEventRecord(c->ev_pb[set], ps));
        c->pdone_st[set] = ps;
        HIPCHK(hipGetLastError());
        return ODO_OK;
    }
    // RANSAC part 1 (prep + first eval launch) finishes most pairs; their PnP
    // starts on its own stream while part 2 evaluates the long pairs, whose
    // PnP runs on a second stream so the pair stream moves on to the next batch
    launch_ransac(st, P.good, P.n_good, P.n_matches, P.matches, xyz, c->kp_cap, 0, c->match_cap, c->rcfg, c->latch,
                  P.pair_valid, 20, nullptr, c->rscr[set], P.best_mask, c->mask_words, P.res, P.T12, n, 1,
                  P.pair_phase);
    HIPCHK(hipEventRecord(c->ev_ra[set], st));
    HIPCHK(hipStreamWaitEvent(c->pnpa, c->ev_ra[set], 0));
    if (!(c->skip & 1))
    launch_pnp(c->pnpa, P.f2_src, xyz, c->kun + b * KC * 2, c->ur + b * KC, nkp, c->kp_cap, 0, c->cal, P.T12,
               P.pair_valid, P.n_matches, 20, P.edges, P.res, P.pnp_mask, n, P.pair_phase, 1);
    HIPCHK(hipEventRecord(c->ev_pa[set], c->pnpa));
    if (!(c->skip & 2))
    launch_ransac(st, P.good, P.n_good, P.n_matches, P.matches, xyz, c->kp_cap, 0, c->match_cap, c->rcfg, c->latch,
                  P.pair_valid, 20, nullptr, c->rscr[set], P.best_mask, c->mask_words, P.res, P.T12, n, 2,
                  P.pair_phase, c->h_open + set);
    tmark(c, 8, st);
    HIPCHK(hipEventRecord(c->ev_rb[set], st));
    HIPCHK(hipStreamWaitEvent(c->pnpb, c->ev_rb[set], 0));
    if (!(c->skip & 1))
    launch_pnp(c->pnpb, P.f2_src, xyz, c->kun + b * KC * 2, c->ur + b * KC, nkp, c->kp_cap, 0, c->cal, P.T12,
               P.pair_valid, P.n_matches, 20, P.edges, P.res, P.pnp_mask, n, P.pair_phase, 0);
    tmark(c, 9, c->pnpb);
    HIPCHK(hipEventRecord(c->ev_pb[set], c->pnpb));
    c->pdone_st[set] = nullptr;  // two streams: wait on both events
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

// n_matches / n_queries of the batch's result records (0 for a pair without a
// previous frame), on the device so the records can be copied out asynchronously
__global__ void k_res_patch(odo_pair_result* __restrict__ res, const int* __restrict__ n_matches,
                            const int* __restrict__ qcnt, int n, int first_valid) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool v = i > 0 || first_valid;
    res[i].n_matches = v ? n_matches[i] : 0;
    res[i].n_queries = v ? qcnt[i] : 0;
}

static int finish_batch(odo_ctx* c, int set, int n, odo_pair_result* h_results) {
    if (!h_results) return ODO_OK;
    int e;
    if ((e = sync_all(c))) return e;
    auto& P = c->pb[set];
    HIPCHK(hipMemcpy(h_results, P.res, n * sizeof(odo_pair_result), hipMemcpyDeviceToHost));
    std::vector<int> nm(n);
    HIPCHK(hipMemcpy(nm.data(), P.n_matches, n * sizeof(int), hipMemcpyDeviceToHost));
    std::vector<int> nq(n);
    HIPCHK(hipMemcpy(nq.data(), c->qcnt[set], n * sizeof(int), hipMemcpyDeviceToHost));
    // n_matches and the kNN-2 query counts into the result records
    for (int i = 0; i < n; i++) {
        h_results[i].n_matches = c->valid_h[i] ? nm[i] : 0;
        h_results[i].n_queries = c->valid_h[i] ? nq[i] : 0;
    }
    return ODO_OK;
}

int odo_track_batch(odo_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, int n, odo_pair_result* h_results) {
    if (!c || !d_bgr || !d_depth || n <= 0 || n > c->maxb) return fail(ODO_ERR_ARG, "bad track args");
    int e;
    // decided before this call queues anything: a not-ready query leaves
    // hipErrorNotReady as the thread's last error, cleared here
    c->latched = false;
    if (ODO_WAIT_DEDUP && c->sched == 5 && c->latch_rec && __atomic_load_n(c->latch_set_h, __ATOMIC_ACQUIRE) != 0) {
        const hipError_t q = hipEventQuery(c->ev_latch);
        if (q == hipSuccess) c->latched = true;
        else if (q == hipErrorNotReady) (void)hipGetLastError();
        else return fail(ODO_ERR_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(q));
    }
    const int s = next_set(c);
    const size_t KC = (size_t)c->kp_cap;
    // ---- extraction stream: set s is free once the pair stages of the batch
    // before the previous one (which read it) are done
    if (c->pre_waited != c->batch_counter && (e = queue_batch_waits(c, c->batch_counter))) return e;
    if (c->knn_gate && c->knn_rec) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_knn, 0));
    tmark(c, 0, c->stream);
    // (the next batch's roll reads this set's last frame on its pair stream,
    // before its PnP: the batch that reuses this set waits for that PnP
    // through PYR_WAIT, which therefore has to lie in [1, NSETS - 1])
    const bool geo_pair = ODO_GEO_PAIR && c->sched == 5 && c->knn_pair && !c->adaptive && !c->adaptive_orb &&
                          !c->timing && !c->host_call && c->ev_geo[0] && c->pyr_wait >= 1 &&
                          c->pyr_wait <= NSETS - 1;
    if (c->has_prev && !geo_pair) {
        // the previous batch's last frame becomes slot 0 (Tracking::mLastFrame);
        // its geometry ran on that batch's pair stream when it took that path
        if (c->geo_rec[c->seq_set]) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_geo[c->seq_set], 0));
        const size_t src = fbase(c, c->seq_set) + c->seq_n, dst = fbase(c, s);
        launch_copy_frame(c->stream, c->kps + src * KC, c->desc + src * KC * 32, c->kun + src * KC * 2,
                          c->xyz + src * KC * 3, c->ur + src * KC, c->nkp + src, c->kps + dst * KC,
                          c->desc + dst * KC * 32, c->kun + dst * KC * 2, c->xyz + dst * KC * 3, c->ur + dst * KC,
                          c->nkp + dst, c->kp_cap);
    }
    // (Round 6 measured ev_xdone completed by the last extraction kernel,
    // hipExtLaunchKernel's stop event, instead of a marker packet: with the
    // runtime's worker-thread dispatch the pair stream's wait on it did not
    // always hold (a batch's kNN-2 started before the previous batch's, seen
    // in the step marks), and the step was no faster. Not kept.)
    c->geo_pair = geo_pair;  // run_extract leaves the geometry out (only for this call)
    c->early_waits = ODO_EARLY_WAIT && c->sched == 5 && !c->adaptive && !c->adaptive_orb;
    e = run_extract(c, s, d_bgr, d_depth, n, 1);
    c->geo_pair = false;
    c->early_waits = false;
    if (e) return e;
    // the kNN-2 stream: the extraction stream, or the side stream (sched 3)
    hipStream_t ks = c->stream;
    if (c->sched == 3) {
        // side stream: the rand() words first (seed-only, they overlap the
        // extraction), then kNN-2 once the batch's descriptors exist
        if (c->pdone_rec[s]) HIPCHK(hipStreamWaitEvent(c->side, c->ev_rb[s], 0));
        launch_ransac_raw(c->side, c->rscr[s], n, c->match_cap, c->mask_words, c->rcfg, (uint64_t)c->cfg.seed,
                          c->pair_counter, nullptr);
        HIPCHK(hipEventRecord(c->ev_xdone[s], c->stream));
        HIPCHK(hipStreamWaitEvent(c->side, c->ev_xdone[s], 0));
        ks = c->side;
    }
    // kNN-2 of the batch's pairs on stream ks (event pair around it in timing mode 2)
    auto knn_on = [&](hipStream_t kst) -> int {
        const size_t b = fbase(c, s);
        uint8_t* desc = c->desc + b * KC * 32;
        int* nkp = c->nkp + b;
        // the query frames' VO landmarks first: kNN-2 runs on their keypoints only
        const float mThDepth = c->cfg.calib.mbf * c->cfg.calib.th_depth / c->cfg.calib.fx;
        launch_vo_lm(kst, c->xyz + b * KC * 3, nkp, c->kp_cap, 0, mThDepth, c->lm_bits[s], c->lm_words, c->qlist[s],
                     c->qcnt[s], n);
        int kt = -1;
        if (c->ktiming) {
            kt = c->kt_next;
            if (c->kt_pending == odo_ctx::KT_RING) {  // slot reused: fold its time first
                int e2;
                if ((e2 = kt_collect(c, kt))) return e2;
                c->kt_pending--;
            }
            HIPCHK(hipEventRecord(c->kt0[kt], kst));
        }
        c->last_knn_set = s;  // odo_knn_replay_time
        c->last_knn_n = n;
        if (!(c->skip & 8)) {
            if (c->knn_mx)
                launch_knn2_mx(kst, desc, nkp, KC * 32, desc + KC * 32, nkp + 1, KC * 32, c->knn_idx[s], c->knn_dist[s],
                               KC, c->kp_cap, n, c->qlist[s], c->qcnt[s], KC, c->knn_mx);
            else
                launch_knn2(kst, desc, nkp, KC * 32, desc + KC * 32, nkp + 1, KC * 32, c->knn_idx[s], c->knn_dist[s],
                            KC, c->kp_cap, n, c->qlist[s], c->qcnt[s], KC, c->knn_split, (size_t)c->maxb * KC);
        }
        if (kt >= 0) {
            HIPCHK(hipEventRecord(c->kt1[kt], kst));
            c->kt_next = (kt + 1) % odo_ctx::KT_RING;
            c->kt_pending++;
        }
        tmark(c, 10, kst);
        if (c->knn_gate) {
            HIPCHK(hipEventRecord(c->ev_knn, kst));
            c->knn_rec = true;
        }
        return ODO_OK;
    };
    // schedule 5 runs kNN-2 at the head of the batch's pair stream (the
    // extraction stream, the critical one, goes on to the next batch)
    const bool knn_pair = c->sched == 5 && c->knn_pair;
    if (!knn_pair && (e = knn_on(ks))) return e;
    if (c->sched == 3) {
        HIPCHK(hipEventRecord(c->ev_raw[s], c->side));
        HIPCHK(hipEventRecord(c->ev_xdone[s], c->side));
    } else if (c->sched == 0) {
        // RANSAC's rand() words (seed-only) at the end of the extraction
        // stream: set s was released (ev_pa/ev_pb) before this batch began
        launch_ransac_raw(c->stream, c->rscr[s], n, c->match_cap, c->mask_words, c->rcfg, (uint64_t)c->cfg.seed,
                          c->pair_counter, nullptr);
        HIPCHK(hipEventRecord(c->ev_xdone[s], c->stream));
        HIPCHK(hipEventRecord(c->ev_raw[s], c->stream));
    } else if (c->sched == 4 || c->sched == 5) {
        // the words at the head of the batch's pair stream; schedule 5
        // alternates two pair streams (each also runs its batch's PnP), so one
        // batch's long RANSAC / PnP overlaps the next batch's pair stages
        if (c->sched == 5) {
            const int q = (int)(c->batch_counter % (uint64_t)c->npstreams);
            c->cur_p = q == 0 ? c->pstream : (q == 1 ? c->pstream2 : c->pstream3);
        } else {
            c->cur_p = c->pstream;
        }
        if (c->pdone_rec[s] && (e = wait_pnp_done(c, c->cur_p, s))) return e;
        HIPCHK(hipEventRecord(c->ev_xdone[s], c->stream));
        launch_ransac_raw(c->cur_p, c->rscr[s], n, c->match_cap, c->mask_words, c->rcfg, (uint64_t)c->cfg.seed,
                          c->pair_counter, nullptr);
        // the words and their reader share the stream: no marker (ODO_WAIT_DEDUP)
        if (!ODO_WAIT_DEDUP) HIPCHK(hipEventRecord(c->ev_raw[s], c->cur_p));
    } else {
        HIPCHK(hipEventRecord(c->ev_xdone[s], c->stream));
        // ---- side stream: RANSAC's rand() words depend on the pair seeds only
        if (c->pdone_rec[s]) HIPCHK(hipStreamWaitEvent(c->side, c->ev_rb[s], 0));
        launch_ransac_raw(c->side, c->rscr[s], n, c->match_cap, c->mask_words, c->rcfg, (uint64_t)c->cfg.seed,
                          c->pair_counter, nullptr);
        HIPCHK(hipEventRecord(c->ev_raw[s], c->side));
    }
    // ---- pair stream
    if (c->sched != 4 && c->sched != 5) c->cur_p = c->pstream;
    HIPCHK(hipStreamWaitEvent(c->cur_p, c->ev_xdone[s], 0));
    if (!(ODO_WAIT_DEDUP && (c->sched == 4 || c->sched == 5))) HIPCHK(hipStreamWaitEvent(c->cur_p, c->ev_raw[s], 0));
    if (geo_pair) {
        // the roll (the previous batch's last frame into slot 0, once that
        // batch's geometry is done) and this batch's geometry, ahead of kNN-2
        const size_t b = fbase(c, s);
        if (c->has_prev) {
            const size_t src = fbase(c, c->seq_set) + c->seq_n, dst = b;
            if (c->geo_rec[c->seq_set]) HIPCHK(hipStreamWaitEvent(c->cur_p, c->ev_geo[c->seq_set], 0));
            launch_copy_frame(c->cur_p, c->kps + src * KC, c->desc + src * KC * 32, c->kun + src * KC * 2,
                              c->xyz + src * KC * 3, c->ur + src * KC, c->nkp + src, c->kps + dst * KC,
                              c->desc + dst * KC * 32, c->kun + dst * KC * 2, c->xyz + dst * KC * 3, c->ur + dst * KC,
                              c->nkp + dst, c->kp_cap);
        }
        launch_kp_geometry(c->cur_p, c->kps + (b + 1) * KC, c->nkp + b + 1, d_depth, (size_t)c->W * c->H, c->W, c->cal,
                           c->kun + (b + 1) * KC * 2, c->xyz + (b + 1) * KC * 3, c->ur + (b + 1) * KC, c->kp_cap, n);
        HIPCHK(hipEventRecord(c->ev_geo[s], c->cur_p));
        c->geo_rec[s] = true;
    } else {
        c->geo_rec[s] = false;
    }
    if (knn_pair && (e = knn_on(c->cur_p))) return e;
    c->valid_h.assign(n, 1);
    c->valid_h[0] = c->has_prev ? 1 : 0;
    if (!(c->skip & 4) && (e = run_pairs(c, s, n))) return e;
    c->pdone_rec[s] = true;
    c->seq_set = s;
    c->seq_n = n;
    c->view_set = s;
    c->last_n = n;
    c->has_prev = true;
    c->pair_counter += (uint64_t)n;
    c->batch_set[c->batch_counter & 7] = s;
    c->batch_counter++;
    if ((e = finish_batch(c, s, n, h_results))) return e;
    return ODO_OK;
}

// odo_track_batch with the result records copied into page-locked host memory
// asynchronously (on the batch's pair stream, after its PnP): no host sync, so
// batches keep streaming; the records are valid after odo_synchronize().
int odo_track_batch_async(odo_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, int n, odo_pair_result* h_results) {
    if (!h_results) return fail(ODO_ERR_ARG, "null results");
    const int first_valid = c && c->has_prev ? 1 : 0;
    int e;
    c->defer_pdone = true;  // the PnP-done events are recorded after the copy below
    e = odo_track_batch(c, d_bgr, d_depth, n, nullptr);
    c->defer_pdone = false;
    if (e) return e;
    const int s = c->view_set;
    auto& P = c->pb[s];
    hipStream_t st = c->cur_p ? c->cur_p : c->pstream;  // the batch's pair stream (its PnP ran there last)
    if ((e = wait_pnp_done(c, st, s))) return e;
    hipLaunchKernelGGL(k_res_patch, dim3((n + 255) / 256), dim3(256), 0, st, P.res, P.n_matches, c->qcnt[s], n,
                       first_valid);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h_results, P.res, (size_t)n * sizeof(odo_pair_result), hipMemcpyDeviceToHost, st));
    // the batch that next reuses set s waits for these events: include the copy
    if (!(ODO_WAIT_DEDUP && c->sched == 5)) HIPCHK(hipEventRecord(c->ev_pa[s], st));
    HIPCHK(hipEventRecord(c->ev_pb[s], st));
    c->pdone_st[s] = st;
    return ODO_OK;
}

// Position the sequence (SURVEY §8(e) frames mode): the next batch's pair p
// gets the global pair index pair_index + p (its per-pair RANSAC seed); with
// keep_prev = 0 the next batch's first frame starts a sequence segment (no
// pair with the previous call's last frame: a rank's halo frame). The latch
// and the ADAPTIVE thresholds are kept.
int odo_seek(odo_ctx* c, uint64_t pair_index, int keep_prev) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    c->pair_counter = pair_index;
    if (!keep_prev) c->has_prev = false;
    return ODO_OK;
}

// Host inputs (main.cpp:93-102 hands Track() images in host memory): the
// upload of this batch goes to staging buffer k on the copy stream and the
// extraction stream waits for it, so it overlaps the compute of the batches
// already queued. Buffer k is rewritten only after the extraction that last
// read it (two batches earlier) is done. The call returns once the host
// buffers have been consumed (the caller may refill them), on the error path
// too; with pinned buffers (odo_host_alloc, or hipHostRegister'ed) the DMA
// engines read them directly, pageable ones are staged by the runtime.
// sparse: only the BGR frames are uploaded and the extraction reads the
// keypoints' depth pixels in place through the mapped pointer (the depth
// buffer stays in use until ev_depth_done, odo_host_depth_query / _wait).
// async_res: the result records stream to page-locked memory as in
// odo_track_batch_async (no host sync).
static int track_host(odo_ctx* c, const uint8_t* bgr, const uint16_t* depth, int n, bool sparse,
                      odo_pair_result* h_results, odo_pair_result* async_res) {
    if (!c || !bgr || !depth || n <= 0 || n > c->maxb) return fail(ODO_ERR_ARG, "bad track args");
    void* dmap = nullptr;
    if (sparse) {
        // only HIP page-locked host memory may be read by a kernel (pageable
        // memory would fault): check the allocation type before taking its
        // device pointer
        hipPointerAttribute_t attr{};
        if (hipPointerGetAttributes(&attr, depth) != hipSuccess || attr.type != hipMemoryTypeHost ||
            hipHostGetDevicePointer(&dmap, (void*)depth, 0) != hipSuccess || !dmap) {
            (void)hipGetLastError();
            return fail(ODO_ERR_ARG, "sparse depth: depth must be page-locked host memory (odo_host_alloc)");
        }
    }
    const int k = c->in_next;
    c->in_next ^= 1;
    if (c->in_used[k]) HIPCHK(hipStreamWaitEvent(c->cstream, c->ev_in_free[k], 0));
    const size_t px = (size_t)n * c->W * c->H;
    HIPCHK(hipMemcpyAsync(c->bgr_in[k], bgr, px * 3, hipMemcpyHostToDevice, c->cstream));
    if (!sparse) HIPCHK(hipMemcpyAsync(c->depth_in[k], depth, px * 2, hipMemcpyHostToDevice, c->cstream));
    HIPCHK(hipEventRecord(c->ev_in_copied[k], c->cstream));
    int e = ODO_OK;
    if (hipStreamWaitEvent(c->stream, c->ev_in_copied[k], 0) != hipSuccess) e = fail(ODO_ERR_DEVICE, "hipStreamWaitEvent");
    const uint16_t* dd = sparse ? (const uint16_t*)dmap : c->depth_in[k];
    c->host_call = true;  // the batch's depth reads stay on the extraction stream (ev_in_free, ev_depth_done)
    if (!e) e = async_res ? odo_track_batch_async(c, c->bgr_in[k], dd, n, async_res)
                          : odo_track_batch(c, c->bgr_in[k], dd, n, nullptr);
    c->host_call = false;
    if (!e) {
        // everything that reads staging buffer k (and a sparse batch's depth
        // frames) is queued on the extraction stream
        if (hipEventRecord(c->ev_in_free[k], c->stream) != hipSuccess) e = fail(ODO_ERR_DEVICE, "hipEventRecord");
        c->in_used[k] = true;
        if (!e && sparse) {
            if (hipEventRecord(c->ev_depth_done, c->stream) != hipSuccess) e = fail(ODO_ERR_DEVICE, "hipEventRecord");
            c->depth_busy = true;
        }
    }
    // the host buffers are free once their copy has landed, whatever happened
    // after the copy was queued
    const hipError_t se = hipEventSynchronize(c->ev_in_copied[k]);
    if (e) return e;
    if (se != hipSuccess) return fail(ODO_ERR_DEVICE, std::string("hipEventSynchronize: ") + hipGetErrorString(se));
    return finish_batch(c, c->view_set, n, h_results);
}

int odo_track_batch_host(odo_ctx* c, const uint8_t* bgr, const uint16_t* depth, int n, odo_pair_result* h_results) {
    return track_host(c, bgr, depth, n, false, h_results, nullptr);
}

int odo_track_batch_host_async(odo_ctx* c, const uint8_t* bgr, const uint16_t* depth, int n,
                               odo_pair_result* h_results) {
    if (!h_results) return fail(ODO_ERR_ARG, "null results");
    return track_host(c, bgr, depth, n, false, nullptr, h_results);
}

int odo_track_batch_host_sparse_depth(odo_ctx* c, const uint8_t* bgr, const uint16_t* depth, int n,
                                      odo_pair_result* h_results) {
    return track_host(c, bgr, depth, n, true, h_results, nullptr);
}

int odo_host_depth_query(odo_ctx* c) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    if (!c->depth_busy) return 0;
    const hipError_t q = hipEventQuery(c->ev_depth_done);
    if (q == hipSuccess) {
        c->depth_busy = false;
        return 0;
    }
    if (q == hipErrorNotReady) return 1;
    return fail(ODO_ERR_DEVICE, std::string("hipEventQuery: ") + hipGetErrorString(q));
}

int odo_host_depth_wait(odo_ctx* c) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    if (!c->depth_busy) return ODO_OK;
    HIPCHK(hipEventSynchronize(c->ev_depth_done));
    c->depth_busy = false;
    return ODO_OK;
}

void* odo_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        fail(ODO_ERR_DEVICE, "hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

int odo_host_free(void* p) {
    if (p) HIPCHK(hipHostFree(p));
    return ODO_OK;
}

int odo_get_frame(odo_ctx* c, int i, orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz, float* u_right, int cap,
                  int* n) {
    if (!c || i < 0 || i >= c->last_n) return fail(ODO_ERR_ARG, "bad frame index");
    int e;
    if ((e = sync_all(c))) return e;
    // frame i of the last batch: slot i+1 of its frame set
    const size_t slot = fbase(c, c->view_set) + i + 1;
    // every array at its full capacity (no round trip for the count first):
    // async copies into the pinned staging buffer, one sync, then the
    // caller's buffers
    const size_t KC = (size_t)c->kp_cap;
    Pack pk;
    const size_t o_n = pk.add(sizeof(int)), o_k = pk.add(KC * sizeof(orb_kp)), o_d = pk.add(KC * 32),
                 o_u = pk.add(KC * 8), o_x = pk.add(KC * 12), o_r = pk.add(KC * 4);
    if ((e = stage_reserve(c, pk.off))) return e;
    uint8_t* h = c->stage_h;
    hipStream_t st = c->stream;
    HIPCHK(hipMemcpyAsync(h + o_n, c->nkp + slot, sizeof(int), hipMemcpyDeviceToHost, st));
    if (kps) HIPCHK(hipMemcpyAsync(h + o_k, c->kps + slot * KC, KC * sizeof(orb_kp), hipMemcpyDeviceToHost, st));
    if (desc) HIPCHK(hipMemcpyAsync(h + o_d, c->desc + slot * KC * 32, KC * 32, hipMemcpyDeviceToHost, st));
    if (kps_un) HIPCHK(hipMemcpyAsync(h + o_u, c->kun + slot * KC * 2, KC * 8, hipMemcpyDeviceToHost, st));
    if (xyz) HIPCHK(hipMemcpyAsync(h + o_x, c->xyz + slot * KC * 3, KC * 12, hipMemcpyDeviceToHost, st));
    if (u_right) HIPCHK(hipMemcpyAsync(h + o_r, c->ur + slot * KC, KC * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    int cnt = 0;
    memcpy(&cnt, h + o_n, sizeof(int));
    *n = cnt;
    const int m = std::max(0, std::min(cnt, cap));
    if (kps) memcpy(kps, h + o_k, (size_t)m * sizeof(orb_kp));
    if (desc) memcpy(desc, h + o_d, (size_t)m * 32);
    if (kps_un) memcpy(kps_un, h + o_u, (size_t)m * 8);
    if (xyz) memcpy(xyz, h + o_x, (size_t)m * 12);
    if (u_right) memcpy(u_right, h + o_r, (size_t)m * 4);
    return cnt > cap ? fail(ODO_ERR_CAPACITY, "cap too small") : ODO_OK;
}

int odo_get_pair(odo_ctx* c, int i, odo_dmatch* matches, int match_cap, int* n_matches, odo_dmatch* good_sorted,
                 int* n_good, uint8_t* ransac_inliers, uint8_t* pnp_inliers, int32_t* f2_src) {
    if (!c || i < 0 || i >= c->last_n) return fail(ODO_ERR_ARG, "bad pair index");
    int e;
    if ((e = sync_all(c))) return e;
    int nm = 0, ng = 0, n2 = 0;
    auto& P = c->pb[c->view_set];
    HIPCHK(hipMemcpy(&nm, P.n_matches + i, sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&ng, P.n_good + i, sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&n2, c->nkp + fbase(c, c->view_set) + i + 1, sizeof(int), hipMemcpyDeviceToHost));
    if (n_matches) *n_matches = nm;
    if (n_good) *n_good = ng;
    std::vector<odo_dmatch> M(std::max(nm, 1));
    HIPCHK(hipMemcpy(M.data(), P.matches + (size_t)i * c->match_cap, nm * sizeof(odo_dmatch), hipMemcpyDeviceToHost));
    if (matches) memcpy(matches, M.data(), std::min(nm, match_cap) * sizeof(odo_dmatch));
    if (good_sorted || ransac_inliers) {
        std::vector<uint64_t> G(std::max(ng, 1));
        HIPCHK(hipMemcpy(G.data(), (uint64_t*)P.good + (size_t)i * c->match_cap, ng * sizeof(uint64_t),
                         hipMemcpyDeviceToHost));
        if (good_sorted)
            for (int k = 0; k < ng && k < match_cap; k++) good_sorted[k] = M[(uint32_t)(G[k] >> 32)];
        if (ransac_inliers) {
            std::vector<uint32_t> bm(c->mask_words);
            HIPCHK(hipMemcpy(bm.data(), P.best_mask + (size_t)i * c->mask_words, c->mask_words * 4,
                             hipMemcpyDeviceToHost));
            for (int k = 0; k < ng && k < match_cap; k++) ransac_inliers[k] = (bm[k >> 5] >> (k & 31)) & 1;
        }
    }
    if (pnp_inliers) HIPCHK(hipMemcpy(pnp_inliers, P.pnp_mask + (size_t)i * c->kp_cap, n2, hipMemcpyDeviceToHost));
    if (f2_src) HIPCHK(hipMemcpy(f2_src, P.f2_src + (size_t)i * c->kp_cap, n2 * sizeof(int32_t), hipMemcpyDeviceToHost));
    return ODO_OK;
}

// levels back to back, rows compacted (the device layout pitches rows to 16 bytes)
static int copy_levels(odo_ctx* c, const uint8_t* dev, uint8_t* out, size_t cap) {
    size_t total = 0;
    for (auto& L : c->lv_h) total += (size_t)L.w * L.h;
    if (cap < total) return fail(ODO_ERR_ARG, "output buffer too small");
    std::vector<uint8_t> buf(c->pyr_size);
    HIPCHK(hipMemcpy(buf.data(), dev, c->pyr_size, hipMemcpyDeviceToHost));
    size_t o = 0;
    for (auto& L : c->lv_h)
        for (int y = 0; y < L.h; y++, o += L.w) memcpy(out + o, buf.data() + L.off + (size_t)y * L.pitch, L.w);
    return (int)o;
}

int odo_debug_pyramid(odo_ctx* c, int i, uint8_t* out, size_t cap) {
    if (!c || i < 0 || i >= c->last_n || !out) return fail(ODO_ERR_ARG, "bad args");
    int e;
    if ((e = sync_all(c))) return e;
    return copy_levels(c, c->pyr + (fbase(c, c->view_set) + i + 1) * c->pyr_size, out, cap);
}

int odo_debug_blur(odo_ctx* c, int i, uint8_t* out, size_t cap) {
    if (!c || i < 0 || i >= c->last_n || !out) return fail(ODO_ERR_ARG, "bad args");
    int e;
    if ((e = sync_all(c))) return e;
    return copy_levels(c, c->blur + (fbase(c, c->view_set) + i + 1) * c->pyr_size, out, cap);
}

int odo_debug_adaptive(odo_ctx* c, int i, int32_t* t_used, double* thresh) {
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    if (!c->adaptive) return fail(ODO_ERR_STATE, "context is not in ADAPTIVE mode");
    if (t_used && (i < 0 || i >= c->last_n)) return fail(ODO_ERR_ARG, "bad frame index");
    int e;
    if ((e = sync_all(c))) return e;
    if (t_used)
        HIPCHK(hipMemcpy(t_used, c->atsel + (size_t)i * c->ad_ncells, c->ad_ncells * sizeof(int),
                         hipMemcpyDeviceToHost));
    if (thresh) HIPCHK(hipMemcpy(thresh, c->athresh, c->ad_ncells * sizeof(double), hipMemcpyDeviceToHost));
    return c->ad_ncells;
}

int odo_set_adaptive_thresholds(odo_ctx* c, const double* thresh, int n) {
    if (!c || !thresh) return fail(ODO_ERR_ARG, "bad args");
    if (!c->adaptive) return fail(ODO_ERR_STATE, "context is not in ADAPTIVE mode");
    if (n != c->ad_ncells) return fail(ODO_ERR_ARG, "threshold count != grid cells");
    int e;
    if ((e = sync_all(c))) return e;
    HIPCHK(hipMemcpy(c->athresh, thresh, n * sizeof(double), hipMemcpyHostToDevice));
    return ODO_OK;
}

int odo_debug_select(odo_ctx* c, const uint32_t* in, int n, int nth, int mode, uint32_t* out, int* n_out) {
    if (!c || n < 0 || (n && (!in || !out)) || !n_out || nth < 0 || (mode != 0 && mode != 1) || (mode == 1 && nth < 1))
        return fail(ODO_ERR_ARG, "bad select args");
    int e;
    if ((e = sync_all(c))) return e;
    if (n == 0) {
        *n_out = 0;
        return ODO_OK;
    }
    if (nth > n) nth = n;
    void* d = nullptr;
    const size_t bytes = (size_t)n * 12 + 16;
    HIPCHK(hipMalloc(&d, bytes));
    uint32_t* A = (uint32_t*)d;
    int* posL = (int*)(A + n);
    int* posR = posL + n;
    int* dn = posR + n;
    hipError_t er = hipMemcpy(A, in, (size_t)n * 4, hipMemcpyHostToDevice);
    if (er == hipSuccess) {
        launch_adapt_select_dbg(c->stream, A, n, nth, mode, posL, posR, dn);
        er = hipStreamSynchronize(c->stream);
    }
    if (er == hipSuccess) er = hipMemcpy(out, A, (size_t)n * 4, hipMemcpyDeviceToHost);
    if (er == hipSuccess) er = hipMemcpy(n_out, dn, sizeof(int), hipMemcpyDeviceToHost);
    hipFree(d);
    if (er != hipSuccess) return fail(ODO_ERR_DEVICE, hipGetErrorString(er));
    return ODO_OK;
}

// Measurement: re-run the most recent batch's kNN-2 launch `reps` times on one
// stream of an otherwise idle device (all streams drained first; same inputs,
// same outputs rewritten) and return the mean launch time from HIP events.
int odo_knn_replay_time(odo_ctx* c, int reps, float* avg_ms) {
    if (!c || !avg_ms || reps <= 0) return fail(ODO_ERR_ARG, "knn_replay_time: bad arguments");
    if (c->last_knn_set < 0) return fail(ODO_ERR_ARG, "knn_replay_time: no batch tracked yet");
    int e;
    if ((e = sync_all(c))) return e;
    // hipGetLastError is sticky per thread: an error left by an earlier call
    // is reported as that, not as a failure of the replay
    const hipError_t pending = hipGetLastError();
    if (pending != hipSuccess)
        return fail(ODO_ERR_DEVICE, std::string("knn_replay_time: HIP error pending from an earlier call: ") +
                                        hipGetErrorString(pending));
    const int s = c->last_knn_set, n = c->last_knn_n;
    const size_t b = fbase(c, s), KC = (size_t)c->kp_cap;
    uint8_t* desc = c->desc + b * KC * 32;
    int* nkp = c->nkp + b;
    hipStream_t st = c->stream;
    auto launch = [&]() {
        if (c->knn_mx)
            launch_knn2_mx(st, desc, nkp, KC * 32, desc + KC * 32, nkp + 1, KC * 32, c->knn_idx[s], c->knn_dist[s], KC,
                           c->kp_cap, n, c->qlist[s], c->qcnt[s], KC, c->knn_mx);
        else
            launch_knn2(st, desc, nkp, KC * 32, desc + KC * 32, nkp + 1, KC * 32, c->knn_idx[s], c->knn_dist[s], KC,
                        c->kp_cap, n, c->qlist[s], c->qcnt[s], KC, c->knn_split, (size_t)c->maxb * KC);
    };
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    launch();  // warm
    HIPCHK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; r++) launch();
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    HIPCHK(hipEventDestroy(e0));
    HIPCHK(hipEventDestroy(e1));
    HIPCHK(hipGetLastError());
    *avg_ms = ms / (float)reps;
    return ODO_OK;
}

int odo_debug_sort(odo_ctx* c, const odo_dmatch* in, int n, odo_dmatch* out) {
    if (!c || n < 0 || (n && (!in || !out))) return fail(ODO_ERR_ARG, "bad sort args");
    if (n > 8192) return fail(ODO_ERR_CAPACITY, "debug sort: at most 8192 elements");
    if (n == 0) return ODO_OK;
    std::vector<uint64_t> el(n);
    for (int i = 0; i < n; i++) {
        if (!(in[i].distance >= 0.f)) return fail(ODO_ERR_ARG, "debug sort: negative/NaN distance");
        uint32_t bits;
        memcpy(&bits, &in[i].distance, 4);
        el[i] = ((uint64_t)(uint32_t)i << 32) | bits;  // SortEl{key = distance bits, val = index}
    }
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, (size_t)n * 8));
    hipError_t e = hipMemcpy(d, el.data(), (size_t)n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess && launch_sort_dbg(c->stream, d, n) != 0) e = hipErrorInvalidValue;
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) e = hipMemcpy(el.data(), d, (size_t)n * 8, hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) return fail(ODO_ERR_DEVICE, std::string("debug sort: ") + hipGetErrorString(e));
    for (int i = 0; i < n; i++) out[i] = in[(uint32_t)(el[i] >> 32)];
    return ODO_OK;
}

static orb_kp unpack_key(uint32_t k) {
    orb_kp r;
    r.x = (float)(k & 0xfff);
    r.y = (float)((k >> 12) & 0xfff);
    r.size = 7.f;
    r.angle = -1.f;
    r.response = (float)(k >> 24);
    r.octave = 0;
    r.class_id = -1;
    return r;
}

int odo_debug_fast(odo_ctx* c, int i, int level, orb_kp* out, int cap, int* n) {
    if (!c || i < 0 || i >= c->last_n || level < 0 || level >= c->nlevels) return fail(ODO_ERR_ARG, "bad args");
    int e;
    if ((e = sync_all(c))) return e;
    const size_t slot = fbase(c, c->view_set) + i + 1;
    const LevelDesc& L = c->lv_h[level];
    const int nc = L.cell_end - L.cell_begin;
    std::vector<int> cnt(nc);
    std::vector<uint32_t> cand((size_t)nc * c->cell_cap);
    HIPCHK(hipMemcpy(cnt.data(), c->cand_cnt + (size_t)slot * c->ncells + L.cell_begin, nc * sizeof(int),
                     hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cand.data(), c->cand + ((size_t)slot * c->ncells + L.cell_begin) * c->cell_cap,
                     cand.size() * 4, hipMemcpyDeviceToHost));
    int m = 0;
    for (int ci = 0; ci < nc; ci++)
        for (int k = 0; k < cnt[ci]; k++) {
            if (m < cap) out[m] = unpack_key(cand[(size_t)ci * c->cell_cap + k]);
            m++;
        }
    *n = m;
    return ODO_OK;
}

int odo_debug_octree(odo_ctx* c, int i, int level, orb_kp* out, int cap, int* n) {
    if (!c || i < 0 || i >= c->last_n || level < 0 || level >= c->nlevels) return fail(ODO_ERR_ARG, "bad args");
    int e;
    if ((e = sync_all(c))) return e;
    const size_t slot = fbase(c, c->view_set) + i + 1;
    int cnt = 0;
    HIPCHK(hipMemcpy(&cnt, c->ocnt + (size_t)slot * c->nlevels + level, sizeof(int), hipMemcpyDeviceToHost));
    std::vector<uint32_t> k(std::max(cnt, 1));
    HIPCHK(hipMemcpy(k.data(), c->okp + ((size_t)slot * c->nlevels + level) * c->okp_stride, cnt * 4,
                     hipMemcpyDeviceToHost));
    for (int j = 0; j < cnt && j < cap; j++) out[j] = unpack_key(k[j]);
    *n = cnt;
    return ODO_OK;
}

int odo_last_timings(odo_ctx* c, float* ms, int cap, const char** names) {
    static const char* kNamesOrb[] = {"gray+pyramid", "fast", "octree", "blur", "finalize", "knn2", "match+sort",
                                      "ransac", "pnp"};
    // ADAPTIVE marks: gray | S map + band survivors | chain + select + assemble | blur L0 | finalize
    static const char* kNamesAd[] = {"gray", "smap+cand", "chain+select", "blur", "finalize", "knn2", "match+sort",
                                     "ransac", "pnp"};
    const char* const* kNames = c && c->adaptive ? kNamesAd : kNamesOrb;
    // stage i spans events (a[i], b[i]): extraction stream 0..5,10; pair stream 6..9
    static const int a[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8}, b[9] = {1, 2, 3, 4, 5, 10, 7, 8, 9};
    if (!c) return fail(ODO_ERR_ARG, "null ctx");
    if (!c->timing) return fail(ODO_ERR_ARG, "stage timing is off (odo_set_timing)");
    int e;
    if ((e = sync_all(c))) return e;
    int m = 0;
    for (int i = 0; i < 9 && i < cap; i++) {
        float t = 0;
        if (hipEventElapsedTime(&t, c->ev[a[i]], c->ev[b[i]]) != hipSuccess) t = -1;
        ms[i] = t;
        if (names) names[i] = kNames[i];
        m++;
    }
    return m;
}

void odo_rng_seed(odo_rng* r, uint32_t seed) {
    // glibc __srandom_r (TYPE_3): Schrage LCG fill, fptr=3, rptr=0, 310 discards
    if (seed == 0) seed = 1;
    r->state[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        long hi = word / 127773, lo = word % 127773;
        long w2 = 16807 * lo - 2836 * hi;
        if (w2 < 0) w2 += 2147483647;
        word = (int32_t)w2;
        r->state[i] = word;
    }
    r->fpos = 3;
    r->rpos = 0;
    for (int k = 0; k < 310; k++) odo_rng_next(r);
}

int32_t odo_rng_next(odo_rng* r) {
    uint32_t val = (uint32_t)r->state[r->fpos] + (uint32_t)r->state[r->rpos];
    r->state[r->fpos] = (int32_t)val;
    int32_t out = (int32_t)(val >> 1);
    if (++r->fpos >= 31) {
        r->fpos = 0;
        ++r->rpos;
    } else if (++r->rpos >= 31) r->rpos = 0;
    return out;
}

}  // extern "C"

// ====================================================================== per-stage entry points
namespace {
// a carve of the calling entry point's arena (no free: the arena owns it)
struct DevBuf {
    void* p = nullptr;
    DevBuf(DevArena& a, size_t bytes) : p(a.take(bytes)) {}
    template <typename T>
    T* as() {
        return (T*)p;
    }
};
#define ARENA_CHECK(a) \
    if ((a).failed) return fail(ODO_ERR_DEVICE, "device scratch allocation failed")

// Ransac::Iterate's inputs after the depth filter, std::sort and the latch
// (ransac.cpp:164-199), uploaded for the single-pair RANSAC kernels.
struct PairRansacInput {
    std::vector<odo_dmatch> good;
    int ng = 0, words = 0, kc = 1;
    RansacCfg cfg{};
};

// returns 0 when RANSAC does not run (too few matches / good matches)
int prepare_pair_ransac(const odo_dmatch* m12, int n12, const float* xyz1, int n1, const float* xyz2, int n2,
                        const odo_ransac_params* p, double* latch, PairRansacInput& in, int match_cap) {
    if (n12 < p->min_inlier_th) return 0;
    in.good.clear();
    in.good.reserve(n12);
    for (int i = 0; i < n12; i++) {
        const odo_dmatch& m = m12[i];
        if (m.queryIdx < 0 || m.queryIdx >= n1 || m.trainIdx < 0 || m.trainIdx >= n2)
            return fail(ODO_ERR_ARG, "match index out of range");
        const float zs = xyz1[3 * m.queryIdx + 2], zt = xyz2[3 * m.trainIdx + 2];
        if (p->check_depth) {
            if (std::isnan(zs) || std::isnan(zt)) continue;
            if (zs <= 0 || zt <= 0) continue;
        }
        in.good.push_back(m);
    }
    if ((int)in.good.size() < p->min_inlier_th) return 0;
    std::sort(in.good.begin(), in.good.end(),
              [](const odo_dmatch& a, const odo_dmatch& b) { return a.distance < b.distance; });
    in.ng = (int)in.good.size();
    if (in.ng > match_cap * 64) return fail(ODO_ERR_CAPACITY, "too many matches");
    if (std::isnan(*latch)) {  // DepthCovariance first-call latch (ransac.cpp:416-421)
        for (const odo_dmatch& m : in.good) {
            const float* o = &xyz1[3 * m.queryIdx];
            const float* tg = &xyz2[3 * m.trainIdx];
            if (o[2] == 0.0f || tg[0] == 0.0f) continue;
            if (std::isnan(o[2]) || std::isnan(tg[2])) continue;
            const double z = (double)o[2];
            const double sd = 0.01 * z * z;
            *latch = sd * sd;
            break;
        }
    }
    in.kc = std::max(std::max(n1, n2), 1);
    in.words = (in.ng + 31) / 32;
    const double cam_angle_x = 58.0 / 180.0 * M_PI, cam_angle_y = 45.0 / 180.0 * M_PI;
    const double rsx = 3 * tan(cam_angle_x / 640.0), rsy = 3 * tan(cam_angle_y / 480.0);
    in.cfg = RansacCfg{p->iterations, p->min_inlier_th, p->max_mahalanobis, p->sample_size, p->check_depth,
                       rsx * rsx, rsy * rsy};
    return 1;
}
}  // namespace

struct HypSession {
    PairRansacInput in;
    int h0 = 0, h1 = 0, active = 0;
    DevArena& arena;  // the context's hyp_arena: this session's buffers until the next session
    explicit HypSession(DevArena& a) : arena(a) {}
    DevBuf *xyz = nullptr, *m = nullptr, *g = nullptr, *ints = nullptr, *latch = nullptr, *rng = nullptr,
           *res = nullptr, *T = nullptr, *scr = nullptr, *bm = nullptr, *phase = nullptr;
    ~HypSession() {
        DevBuf* b[] = {xyz, m, g, ints, latch, rng, res, T, scr, bm, phase};
        for (DevBuf* x : b) delete x;
    }
};
static void free_hyp_session(HypSession* h) { delete h; }

extern "C" {

int odo_extract(odo_ctx* c, const uint8_t* img, int channels, const uint16_t* depth, orb_kp* kps, uint8_t* desc,
                float* kps_un, float* xyz, float* u_right, int cap, int* n) {
    if (!c || !img || (channels != 1 && channels != 3) || !n) return fail(ODO_ERR_ARG, "bad extract args");
    int e0;
    if ((e0 = sync_all(c))) return e0;
    hipStream_t st = c->stream;
    const size_t npix = (size_t)c->W * c->H;
    const int set = next_set(c);
    const int slot = 1;
    if (depth) HIPCHK(hipMemcpyAsync(c->depth_in[0], depth, npix * 2, hipMemcpyHostToDevice, st));
    else HIPCHK(hipMemsetAsync(c->depth_in[0], 0, npix * 2, st));
    if (channels == 3) {
        HIPCHK(hipMemcpyAsync(c->bgr_in[0], img, npix * 3, hipMemcpyHostToDevice, st));
        tmark(c, 0, st);
        int e = run_extract(c, set, c->bgr_in[0], c->depth_in[0], 1, slot);
        if (e) return e;
    } else {
        // ORBextractor::operator() on a gray image: level 0 = the image itself
        HIPCHK(hipMemcpy2DAsync(c->pyr + (fbase(c, set) + slot) * c->pyr_size, c->lv_h[0].pitch, img, c->W, c->W, c->H,
                                hipMemcpyHostToDevice, st));
        tmark(c, 0, st);
        int e = run_extract_from_gray(c, set, c->depth_in[0], 1, slot);
        if (e) return e;
    }
    c->view_set = set;
    c->last_n = 1;
    return odo_get_frame(c, 0, kps, desc, kps_un, xyz, u_right, cap, n);
}

int odo_knn2_hamming(odo_ctx* c, const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx, int32_t* dist) {
    if (!c || nq < 0 || nt < 0 || (nq && !q) || (nt && !t) || !idx || !dist) return fail(ODO_ERR_ARG, "bad knn args");
    if (nq == 0) return ODO_OK;
    if (nq > (1 << 20) || nt > (1 << 20)) return fail(ODO_ERR_CAPACITY, "knn2: at most 2^20 descriptors");
    hipStream_t st = c->stream;
    DevArena& A = c->arena;
    A.begin();
    // one packed upload (descriptors + counts) and one packed download
    Pack pk;
    const size_t o_q = pk.add((size_t)nq * 32), o_t = pk.add((size_t)std::max(nt, 1) * 32), o_n = pk.add(2 * sizeof(int));
    const size_t in_bytes = pk.off;
    const size_t o_i = pk.add((size_t)nq * sizeof(int2)), o_d = pk.add((size_t)nq * sizeof(int2));
    int e;
    if ((e = stage_reserve(c, pk.off))) return e;
    DevBuf dall(A, pk.off);
    ARENA_CHECK(A);
    uint8_t* h = c->stage_h;
    memcpy(h + o_q, q, (size_t)nq * 32);
    if (nt) memcpy(h + o_t, t, (size_t)nt * 32);
    const int cnt[2] = {nq, nt};
    memcpy(h + o_n, cnt, sizeof(cnt));
    HIPCHK(hipMemcpyAsync(dall.p, h, in_bytes, hipMemcpyHostToDevice, st));
    uint8_t* db = dall.as<uint8_t>();
    const DevView dq{db + o_q}, dt{db + o_t}, dn{db + o_n}, di{db + o_i}, dd{db + o_d};
    if (c->knn_mx && nt <= 8192)  // the packed key holds a 13-bit train index
        launch_knn2_mx(st, dq.as<uint8_t>(), dn.as<int>(), 0, dt.as<uint8_t>(), dn.as<int>() + 1, 0, di.as<int2>(),
                       dd.as<int2>(), 0, nq, 1, nullptr, nullptr, 0, c->knn_mx);
    else
        launch_knn2(st, dq.as<uint8_t>(), dn.as<int>(), 0, dt.as<uint8_t>(), dn.as<int>() + 1, 0, di.as<int2>(),
                    dd.as<int2>(), 0, nq, 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h + o_i, db + o_i, pk.off - o_i, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    memcpy(idx, h + o_i, (size_t)nq * 8);
    memcpy(dist, h + o_d, (size_t)nq * 8);
    return ODO_OK;
}

int odo_ransac(odo_ctx* c, const odo_dmatch* m12, int n12, const float* xyz1, int n1, const float* xyz2, int n2,
               const odo_ransac_params* p, odo_rng* rng, double* latch, float T12[16], float* rmse,
               odo_dmatch* inliers, int* n_inliers, int* ok) {
    if (!c || !p || !rng || !latch || !T12 || !rmse || !n_inliers || !ok || n12 < 0 || (n12 && !m12))
        return fail(ODO_ERR_ARG, "bad ransac args");
    // Iterate() resets its outputs first (ransac.cpp:157-159)
    for (int i = 0; i < 16; i++) T12[i] = (i % 5 == 0) ? 1.f : 0.f;
    *rmse = 1e6f;
    *n_inliers = 0;
    *ok = 0;
    if (n12 < p->min_inlier_th) return ODO_OK;
    // depth filter (ransac.cpp:175-189) and std::sort by distance (ransac.cpp:199)
    std::vector<odo_dmatch> good;
    good.reserve(n12);
    for (int i = 0; i < n12; i++) {
        const odo_dmatch& m = m12[i];
        if (m.queryIdx < 0 || m.queryIdx >= n1 || m.trainIdx < 0 || m.trainIdx >= n2)
            return fail(ODO_ERR_ARG, "match index out of range");
        const float zs = xyz1[3 * m.queryIdx + 2], zt = xyz2[3 * m.trainIdx + 2];
        if (p->check_depth) {
            if (std::isnan(zs) || std::isnan(zt)) continue;
            if (zs <= 0 || zt <= 0) continue;
        }
        good.push_back(m);
    }
    if ((int)good.size() < p->min_inlier_th) return ODO_OK;
    std::sort(good.begin(), good.end(), [](const odo_dmatch& a, const odo_dmatch& b) { return a.distance < b.distance; });
    const int ng = (int)good.size();
    if (ng > c->match_cap * 64) return fail(ODO_ERR_CAPACITY, "too many matches");
    // DepthCovariance first-call latch (ransac.cpp:416-421)
    if (std::isnan(*latch)) {
        for (const odo_dmatch& m : good) {
            const float* o = &xyz1[3 * m.queryIdx];
            const float* tg = &xyz2[3 * m.trainIdx];
            if (o[2] == 0.0f || tg[0] == 0.0f) continue;
            if (std::isnan(o[2]) || std::isnan(tg[2])) continue;
            const double z = (double)o[2];
            const double sd = 0.01 * z * z;
            *latch = sd * sd;
            break;
        }
    }
    hipStream_t st = c->stream;
    const int kc = std::max(std::max(n1, n2), 1);
    const int words = (ng + 31) / 32;
    DevArena& A = c->arena;
    A.begin();
    const double cam_angle_x = 58.0 / 180.0 * M_PI, cam_angle_y = 45.0 / 180.0 * M_PI;
    const double rsx = 3 * tan(cam_angle_x / 640.0), rsy = 3 * tan(cam_angle_y / 480.0);
    RansacCfg cfg{p->iterations, p->min_inlier_th, p->max_mahalanobis, p->sample_size, p->check_depth, rsx * rsx,
                  rsy * rsy};
    // inputs packed into the pinned staging buffer, one upload; the outputs
    // (result record, inlier mask, rand() state) are adjacent, one download
    Pack pk;
    const size_t o_xyz = pk.add((size_t)2 * kc * 12), o_m = pk.add((size_t)ng * sizeof(odo_dmatch)),
                 o_g = pk.add((size_t)ng * 8), o_int = pk.add(4 * sizeof(int)), o_latch = pk.add(sizeof(double));
    const size_t o_rng = pk.add(sizeof(odo_rng));
    const size_t in_bytes = pk.off;
    const size_t o_res = pk.add(sizeof(odo_pair_result)), o_bm = pk.add((size_t)words * 4);
    const size_t all_bytes = pk.off;
    int e0;
    if ((e0 = stage_reserve(c, all_bytes))) return e0;
    DevBuf dall(A, all_bytes), dT(A, 16 * sizeof(float)), dgp(A, ransac_scratch_bytes(1, ng, words, cfg));
    ARENA_CHECK(A);
    uint8_t* h = c->stage_h;
    memcpy(h + o_xyz, xyz1, (size_t)n1 * 12);
    memcpy(h + o_xyz + (size_t)kc * 12, xyz2, (size_t)n2 * 12);
    memcpy(h + o_m, good.data(), (size_t)ng * sizeof(odo_dmatch));
    uint64_t* gl = reinterpret_cast<uint64_t*>(h + o_g);
    for (int k = 0; k < ng; k++) {
        uint32_t bits;
        memcpy(&bits, &good[k].distance, 4);
        gl[k] = ((uint64_t)(uint32_t)k << 32) | bits;
    }
    const int ints[4] = {ng, ng, 1, 0};  // n_good, n_matches, pair_valid
    memcpy(h + o_int, ints, sizeof(ints));
    memcpy(h + o_latch, latch, sizeof(double));
    memcpy(h + o_rng, rng, sizeof(odo_rng));
    HIPCHK(hipMemcpyAsync(dall.p, h, in_bytes, hipMemcpyHostToDevice, st));
    uint8_t* db = dall.as<uint8_t>();
    const DevView dxyz{db + o_xyz}, dm{db + o_m}, dg{db + o_g}, dint{db + o_int}, dlatch{db + o_latch},
        drng{db + o_rng}, dres{db + o_res}, dbm{db + o_bm};
    launch_ransac_raw(st, dgp.p, 1, ng, words, cfg, 0, 0, drng.as<odo_rng>());
    launch_ransac(st, dg.p, dint.as<int>(), dint.as<int>() + 1, dm.as<odo_dmatch>(), dxyz.as<float>(), kc, 0, ng, cfg,
                  dlatch.as<double>(), dint.as<int>() + 2, 0, drng.as<odo_rng>(), dgp.p, dbm.as<uint32_t>(),
                  words, dres.as<odo_pair_result>(), dT.as<float>(), 1);
    HIPCHK(hipGetLastError());
    // rng (updated in place) .. the mask: one contiguous download
    HIPCHK(hipMemcpyAsync(h + o_rng, db + o_rng, all_bytes - o_rng, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    odo_pair_result r;
    memcpy(&r, h + o_res, sizeof(r));
    memcpy(rng, h + o_rng, sizeof(odo_rng));
    const uint32_t* bm = reinterpret_cast<const uint32_t*>(h + o_bm);
    memcpy(T12, r.T12, sizeof(r.T12));
    *rmse = r.rmse;
    int k2 = 0;
    for (int k = 0; k < ng; k++)
        if ((bm[k >> 5] >> (k & 31)) & 1) {
            if (inliers) inliers[k2] = good[k];
            k2++;
        }
    *n_inliers = k2;
    *ok = r.ransac_ok;
    return ODO_OK;
}

// Hypotheses mode, shared by the host and the device exchange: a new session
// over the pair, its samples for all H hypotheses and the evaluation of
// [h0, h1) queued on the context's stream (no fold). *active = 0 when
// Iterate returns before sampling (too few matches).
static int hyps_launch(odo_ctx* c, const odo_dmatch* m12, int n12, const float* xyz1, int n1, const float* xyz2,
                       int n2, const odo_ransac_params* p, const odo_rng* rng, double* latch, int h0, int h1,
                       int* n_good, int* active) {
    free_hyp_session(c->hs);
    c->hs = new HypSession(c->hyp_arena);
    HypSession& S = *c->hs;
    S.h0 = h0;
    S.h1 = h1;
    *n_good = 0;
    *active = 0;
    const int r = prepare_pair_ransac(m12, n12, xyz1, n1, xyz2, n2, p, latch, S.in, c->match_cap);
    if (r < 0) return r;
    if (r == 0) return ODO_OK;  // Iterate returns before the loop (too few matches)
    S.active = 1;
    *active = 1;
    PairRansacInput& in = S.in;
    const int ng = in.ng, kc = in.kc;
    *n_good = ng;
    hipStream_t st = c->stream;
    DevArena& A = S.arena;
    // the previous session's kernels (queued asynchronously by _dev / _finish)
    // may still read the arena that begin() may free and replace
    HIPCHK(hipStreamSynchronize(st));
    A.begin();
    S.xyz = new DevBuf(A, (size_t)2 * kc * 3 * sizeof(float));
    S.m = new DevBuf(A, (size_t)ng * sizeof(odo_dmatch));
    S.g = new DevBuf(A, (size_t)ng * 8);
    S.ints = new DevBuf(A, 4 * sizeof(int));
    S.latch = new DevBuf(A, sizeof(double));
    S.rng = new DevBuf(A, sizeof(odo_rng));
    S.res = new DevBuf(A, sizeof(odo_pair_result));
    S.T = new DevBuf(A, 16 * sizeof(float));
    S.scr = new DevBuf(A, ransac_scratch_bytes(1, ng, in.words, in.cfg));
    S.bm = new DevBuf(A, (size_t)in.words * 4);
    S.phase = new DevBuf(A, 2 * sizeof(int));
    ARENA_CHECK(A);
    std::vector<uint64_t> gl(ng);
    for (int k = 0; k < ng; k++) {
        uint32_t bits;
        memcpy(&bits, &in.good[k].distance, 4);
        gl[k] = ((uint64_t)(uint32_t)k << 32) | bits;
    }
    const int ints[4] = {ng, ng, 1, 0};
    const int range[2] = {h0, h1};
    // the inputs packed in page-locked memory in their device order (the
    // arena hands out consecutive 256-B aligned sections, as Pack does): one
    // DMA instead of seven pageable copies. The previous session's upload
    // must have left the buffer before it is refilled.
    Pack pk;
    const size_t o_xyz = pk.add((size_t)2 * kc * 3 * sizeof(float)), o_m = pk.add((size_t)ng * sizeof(odo_dmatch)),
                 o_g = pk.add((size_t)ng * 8), o_int = pk.add(4 * sizeof(int)), o_lat = pk.add(sizeof(double)),
                 o_rng = pk.add(sizeof(odo_rng));
    const size_t up = o_rng + sizeof(odo_rng);
    if ((uint8_t*)S.rng->p - (uint8_t*)S.xyz->p != (ptrdiff_t)o_rng)
        return fail(ODO_ERR_STATE, "hyps: arena sections not contiguous");
    if (c->hyp_up_rec) HIPCHK(hipEventSynchronize(c->hyp_up));
    if (up > c->hyp_stage_cap) {
        if (c->hyp_stage_h) (void)hipHostFree(c->hyp_stage_h);
        c->hyp_stage_h = nullptr;
        c->hyp_stage_cap = 0;
        const size_t cap = std::max(up, (size_t)1 << 20);
        if (hipHostMalloc((void**)&c->hyp_stage_h, cap, hipHostMallocDefault) != hipSuccess)
            return fail(ODO_ERR_DEVICE, "hipHostMalloc (hypotheses staging) failed");
        c->hyp_stage_cap = cap;
    }
    if (!c->hyp_up) HIPCHK(hipEventCreateWithFlags(&c->hyp_up, ODO_SYNC_EVENT_FLAGS));
    uint8_t* hb = c->hyp_stage_h;
    memcpy(hb + o_xyz, xyz1, (size_t)n1 * 12);
    memcpy(hb + o_xyz + (size_t)kc * 12, xyz2, (size_t)n2 * 12);
    memcpy(hb + o_m, in.good.data(), (size_t)ng * sizeof(odo_dmatch));
    memcpy(hb + o_g, gl.data(), (size_t)ng * 8);
    memcpy(hb + o_int, ints, sizeof(ints));
    memcpy(hb + o_lat, latch, sizeof(double));
    memcpy(hb + o_rng, rng, sizeof(odo_rng));
    HIPCHK(hipMemcpyAsync(S.xyz->p, hb, up, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(c->hyp_up, st));
    c->hyp_up_rec = true;
    // the part-3 launch reads its range from host memory before returning
    int* hrange = const_cast<int*>(range);
    launch_ransac_raw(st, S.scr->p, 1, ng, in.words, in.cfg, 0, 0, S.rng->as<odo_rng>());
    launch_ransac(st, S.g->p, S.ints->as<int>(), S.ints->as<int>() + 1, S.m->as<odo_dmatch>(), S.xyz->as<float>(),
                  kc, 0, ng, in.cfg, S.latch->as<double>(), S.ints->as<int>() + 2, 0, S.rng->as<odo_rng>(), S.scr->p,
                  S.bm->as<uint32_t>(), in.words, S.res->as<odo_pair_result>(), S.T->as<float>(), 1, 3, hrange);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

int odo_ransac_hyps(odo_ctx* c, const odo_dmatch* m12, int n12, const float* xyz1, int n1, const float* xyz2, int n2,
                    const odo_ransac_params* p, const odo_rng* rng, double* latch, int h0, int h1,
                    odo_hyp_summary* out, int* n_good) {
    if (!c || !p || !rng || !latch || !n_good || n12 < 0 || (n12 && !m12) || h0 < 0 || h1 < h0 ||
        h1 > std::max(p->iterations, 0) || (h1 > h0 && !out))
        return fail(ODO_ERR_ARG, "bad ransac_hyps args");
    for (int h = 0; h < h1 - h0; h++) out[h] = odo_hyp_summary{1e6, 0, 0, {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}};
    int active = 0;
    const int e = hyps_launch(c, m12, n12, xyz1, n1, xyz2, n2, p, rng, latch, h0, h1, n_good, &active);
    if (e || !active) return e;
    HypSession& S = *c->hs;
    PairRansacInput& in = S.in;
    hipStream_t st = c->stream;
    if (h1 > h0) {
        std::vector<double> err(h1 - h0);
        std::vector<int> cnt(h1 - h0);
        std::vector<float> T((size_t)(h1 - h0) * 12);
        ransac_read_hyps(st, S.scr->p, in.ng, in.words, in.cfg, h0, h1, err.data(), cnt.data(), T.data());
        HIPCHK(hipGetLastError());
        for (int h = 0; h < h1 - h0; h++) {
            out[h].err = err[h];
            out[h].cnt = cnt[h];
            memcpy(out[h].T, &T[(size_t)h * 12], 48);
        }
    }
    HIPCHK(hipStreamSynchronize(st));
    return ODO_OK;
}

int odo_ransac_hyps_dev(odo_ctx* c, const odo_dmatch* m12, int n12, const float* xyz1, int n1, const float* xyz2,
                        int n2, const odo_ransac_params* p, const odo_rng* rng, double* latch, int h0, int h1,
                        void* d_block, int* n_good) {
    if (!c || !p || !rng || !latch || !n_good || n12 < 0 || (n12 && !m12) || h0 < 0 || h1 < h0 ||
        h1 > std::max(p->iterations, 0) || (h1 > h0 && !d_block))
        return fail(ODO_ERR_ARG, "bad ransac_hyps_dev args");
    int active = 0;
    const int e = hyps_launch(c, m12, n12, xyz1, n1, xyz2, n2, p, rng, latch, h0, h1, n_good, &active);
    if (e) return e;
    hipStream_t st = c->stream;
    if (!active) {
        // no sampling: the default summaries (the fold returns before them)
        if (h1 > h0) {
            // queued on the context's stream behind its earlier work; the
            // host vector dies at return, so this path synchronises (odo.h)
            std::vector<odo_hyp_summary> d(h1 - h0, odo_hyp_summary{1e6, 0, 0, {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}});
            HIPCHK(hipMemcpyAsync(d_block, d.data(), d.size() * sizeof(odo_hyp_summary), hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        return ODO_OK;
    }
    HypSession& S = *c->hs;
    ransac_export_hyps(st, S.scr->p, S.in.ng, S.in.words, S.in.cfg, h0, h1, d_block);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

int odo_ransac_fold(const odo_hyp_summary* all, int H, int n_good, const odo_ransac_params* p,
                    odo_ransac_fold_result* r) {
    if (!p || !r || H < 0 || (H && !all)) return fail(ODO_ERR_ARG, "bad fold args");
    // ransac.cpp:201-249: hypothesis j is the j-th visited iteration; n += 10
    // skips do not consume samples, so the fold walks the summaries in order
    *r = odo_ransac_fold_result{-1, 0, 0, 0, 1e6f, n_good, {0, 0}};
    if (n_good < p->min_inlier_th || n_good < p->sample_size) return ODO_OK;
    const unsigned minInl = (unsigned)p->min_inlier_th;
    int n = 0, best = 0;
    float rmse = 1e6f;
    for (int pos = 0; pos < H && n < p->iterations; pos++) {
        const unsigned rc = (unsigned)all[pos].cnt;
        const double re = all[pos].err;
        r->visited++;
        bool brk = false;
        if (rc > 0) {
            r->valid++;
            if (re <= (double)rmse && rc >= (unsigned)best && rc >= minInl) {
                rmse = (float)re;
                best = (int)rc;
                r->best_h = pos;
                if (rc > n_good * 0.5) n += 10;
                if (rc > n_good * 0.75) n += 10;
                if (rc > n_good * 0.8) brk = true;
            }
        }
        n++;
        if (brk) break;
    }
    r->rmse = rmse;
    r->n_inliers = best;
    return ODO_OK;
}

int odo_ransac_hyps_finish(odo_ctx* c, const odo_ransac_fold_result* r, odo_rng* rng, float T12[16], float* rmse,
                           odo_dmatch* inliers, int* n_inliers, int* ok, int* owner) {
    if (!c || !r || !rng || !T12 || !rmse || !n_inliers || !ok || !owner) return fail(ODO_ERR_ARG, "bad finish args");
    if (!c->hs) return fail(ODO_ERR_STATE, "no odo_ransac_hyps call to finish");
    HypSession& S = *c->hs;
    for (int i = 0; i < 16; i++) T12[i] = (i % 5 == 0) ? 1.f : 0.f;
    *rmse = 1e6f;
    *n_inliers = 0;
    *ok = 0;
    *owner = 1;
    if (!S.active) return ODO_OK;  // Iterate returned before sampling: rng untouched
    PairRansacInput& in = S.in;
    *owner = (r->best_h < 0 || (r->best_h >= S.h0 && r->best_h < S.h1)) ? 1 : 0;
    hipStream_t st = c->stream;
    HIPCHK(hipMemcpyAsync(S.rng->p, rng, sizeof(odo_rng), hipMemcpyHostToDevice, st));
    launch_ransac_finish(st, S.scr->p, in.ng, in.words, in.cfg, S.latch->as<double>(), S.rng->as<odo_rng>(),
                         S.bm->as<uint32_t>(), S.res->as<odo_pair_result>(), S.T->as<float>(), r->best_h, r->visited,
                         r->valid, r->n_inliers, r->rmse);
    HIPCHK(hipGetLastError());
    odo_pair_result pr;
    std::vector<uint32_t> bm(in.words);
    HIPCHK(hipMemcpyAsync(&pr, S.res->p, sizeof(pr), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(bm.data(), S.bm->p, (size_t)in.words * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(rng, S.rng->p, sizeof(odo_rng), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (!*owner) return ODO_OK;
    memcpy(T12, pr.T12, sizeof(pr.T12));
    *rmse = pr.rmse;
    int k2 = 0;
    for (int k = 0; k < in.ng; k++)
        if ((bm[k >> 5] >> (k & 31)) & 1) {
            if (inliers) inliers[k2] = in.good[k];
            k2++;
        }
    *n_inliers = k2;
    *ok = pr.ransac_ok;
    return ODO_OK;
}

int odo_ransac_fold_dev(odo_ctx* c, const void* d_all, int H, void* d_fold) {
    if (!c || !d_fold || H < 0 || (H && !d_all)) return fail(ODO_ERR_ARG, "bad fold_dev args");
    if (!c->hs) return fail(ODO_ERR_STATE, "no odo_ransac_hyps_dev call to fold");
    const HypSession& S = *c->hs;
    const int ng = S.active ? S.in.ng : 0;
    const RansacCfg& k = S.in.cfg;
    launch_hyp_fold(c->stream, d_all, H, S.active ? k.iterations : 0, ng, S.active ? k.min_inlier_th : 1,
                    S.active ? k.sample_size : 1, (odo_ransac_fold_result*)d_fold);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

int odo_ransac_hyps_payload_words(odo_ctx* c) {
    if (!c || !c->hs) return fail(ODO_ERR_STATE, "no odo_ransac_hyps_dev session");
    return hyp_payload_words(c->hs->active ? c->hs->in.ng : 0);
}

int odo_ransac_hyps_finish_dev(odo_ctx* c, const void* d_fold, int rank0, void* d_payload, int payload_words) {
    if (!c || !d_fold || !d_payload) return fail(ODO_ERR_ARG, "bad finish_dev args");
    if (!c->hs) return fail(ODO_ERR_STATE, "no odo_ransac_hyps_dev call to finish");
    HypSession& S = *c->hs;
    const int ng = S.active ? S.in.ng : 0;
    if (payload_words < hyp_payload_words(ng)) return fail(ODO_ERR_CAPACITY, "hyps payload too small");
    hipStream_t st = c->stream;
    if (!S.active) {
        // Iterate returned before sampling: rank 0 reports the reset outputs
        // (T = I, rmse 1e6, not ok), the rand() state is untouched
        std::vector<int> w(payload_words, 0);
        if (rank0) {
            for (int i = 0; i < 16; i++) {
                const float v = (i % 5 == 0) ? 1.f : 0.f;
                memcpy(&w[i], &v, 4);
            }
            const float r = 1e6f;
            memcpy(&w[16], &r, 4);
        }
        HIPCHK(hipMemcpyAsync(d_payload, w.data(), w.size() * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));  // w dies at return (odo.h: this path synchronises)
        return ODO_OK;
    }
    launch_hyp_finish(st, S.scr->p, S.in.ng, S.in.words, S.in.cfg, S.latch->as<double>(), S.rng->as<odo_rng>(),
                      S.bm->as<uint32_t>(), S.res->as<odo_pair_result>(), S.T->as<float>(),
                      (const odo_ransac_fold_result*)d_fold, S.h0, S.h1, rank0, S.m->as<odo_dmatch>(), ng,
                      (int*)d_payload, payload_words);
    HIPCHK(hipGetLastError());
    return ODO_OK;
}

int odo_ransac_hyps_result(odo_ctx* c, const void* d_payload, odo_rng* rng, float T12[16], float* rmse,
                           odo_dmatch* inliers, int* n_inliers, int* ok, int* visited) {
    if (!c || !d_payload || !rng || !T12 || !rmse || !n_inliers || !ok || !visited)
        return fail(ODO_ERR_ARG, "bad hyps_result args");
    if (!c->hs) return fail(ODO_ERR_STATE, "no odo_ransac_hyps_dev session");
    HypSession& S = *c->hs;
    const int ng = S.active ? S.in.ng : 0;
    const int words = hyp_payload_words(ng);
    std::vector<int> w(words);
    hipStream_t st = c->stream;
    HIPCHK(hipMemcpyAsync(w.data(), d_payload, (size_t)words * 4, hipMemcpyDeviceToHost, st));
    if (S.active) HIPCHK(hipMemcpyAsync(rng, S.rng->p, sizeof(odo_rng), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    memcpy(T12, w.data(), 64);
    memcpy(rmse, &w[16], 4);
    *ok = w[17];
    *n_inliers = w[18];
    *visited = w[19];
    if (*n_inliers < 0 || *n_inliers > ng) return fail(ODO_ERR_STATE, "hyps payload: bad inlier count");
    if (inliers && *n_inliers) memcpy(inliers, &w[32], (size_t)*n_inliers * sizeof(odo_dmatch));
    return ODO_OK;
}

int odo_pnp_motion_ba(odo_ctx* c, const float* Xw, const float* obs, int n, const odo_calib* calib,
                      const float Tcw_init[16], float Tcw_out[16], uint8_t* outlier, int* n_inliers) {
    if (!c || n < 0 || (n && (!Xw || !obs)) || !Tcw_init || !Tcw_out || !n_inliers) return fail(ODO_ERR_ARG, "bad pnp args");
    hipStream_t st = c->stream;
    const int kc = std::max(n, 1);
    DevArena& A = c->arena;
    A.begin();
    // inputs packed into the pinned staging buffer, one upload; the result
    // record and the inlier mask adjacent, one download
    Pack pk;
    const size_t o_x = pk.add((size_t)kc * 12), o_kun = pk.add((size_t)2 * kc * 8), o_ur = pk.add((size_t)2 * kc * 4),
                 o_src = pk.add((size_t)kc * 4), o_int = pk.add(4 * sizeof(int)), o_T = pk.add(16 * 4);
    const size_t in_bytes = pk.off;
    const size_t o_res = pk.add(sizeof(odo_pair_result)), o_mask = pk.add((size_t)kc);
    const size_t all_bytes = pk.off;
    int e0;
    if ((e0 = stage_reserve(c, all_bytes))) return e0;
    DevBuf dall(A, all_bytes), dedges(A, (size_t)kc * pnp_edge_bytes());
    ARENA_CHECK(A);
    uint8_t* h = c->stage_h;
    float* kun = reinterpret_cast<float*>(h + o_kun) + 2 * kc;  // slot 1 of the two-slot layout
    float* ur = reinterpret_cast<float*>(h + o_ur) + kc;
    int32_t* src = reinterpret_cast<int32_t*>(h + o_src);
    if (n) memcpy(h + o_x, Xw, (size_t)n * 12);
    for (int i = 0; i < n; i++) {
        kun[2 * i] = obs[3 * i];
        kun[2 * i + 1] = obs[3 * i + 1];
        ur[i] = obs[3 * i + 2];
        src[i] = i;
    }
    const int ints[4] = {0, n, 1, 1 << 30};  // nkp[slot0], nkp[slot1], pair_valid, n_matches
    memcpy(h + o_int, ints, sizeof(ints));
    memcpy(h + o_T, Tcw_init, 64);
    HIPCHK(hipMemcpyAsync(dall.p, h, in_bytes, hipMemcpyHostToDevice, st));
    uint8_t* db = dall.as<uint8_t>();
    const DevView dx{db + o_x}, dkun{db + o_kun}, dur{db + o_ur}, dsrc{db + o_src}, dint{db + o_int}, dT{db + o_T},
        dres{db + o_res}, dmask{db + o_mask};
    const odo_calib& k = calib ? *calib : c->cfg.calib;
    FrameCalib cal{k.fx, k.fy, k.cx, k.cy, k.k1, k.k2, k.p1, k.p2, k.k3, k.depth_factor, k.mbf, 1.0f / k.fx, 1.0f / k.fy};
    launch_pnp(st, dsrc.as<int32_t>(), dx.as<float>(), dkun.as<float>(), dur.as<float>(), dint.as<int>(), kc, 0, cal,
               dT.as<float>(), dint.as<int>() + 2, dint.as<int>() + 3, 0, dedges.p, dres.as<odo_pair_result>(),
               dmask.as<uint8_t>(), 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h + o_res, db + o_res, all_bytes - o_res, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    odo_pair_result r;
    memcpy(&r, h + o_res, sizeof(r));
    const uint8_t* mask = h + o_mask;
    memcpy(Tcw_out, r.Tcw, 64);
    *n_inliers = r.pnp_inliers;
    if (outlier)
        for (int i = 0; i < n; i++) outlier[i] = mask[i] ? 0 : 1;
    return ODO_OK;
}

// PnPRansac::Compute over nprob problems (problem p = points [offs[p], offs[p+1])),
// one launch chain for the whole batch.
static int pnp_ransac_run(odo_ctx* c, const float* Xw, const float* uv, const int32_t* offs, int nprob,
                          const odo_calib* calib, int iterations, float reproj_err, double confidence,
                          odo_pnp_ransac_result* res, uint8_t* inlier_mask, int32_t* good_counts) {
    // ptsetreg.cpp run(): CV_Assert(confidence > 0 && confidence < 1); niters = MAX(maxIters, 1)
    if (!(confidence > 0.0 && confidence < 1.0)) return fail(ODO_ERR_ARG, "confidence must be in (0, 1)");
    const int H = std::max(iterations, 1);
    if (offs[0] != 0) return fail(ODO_ERR_ARG, "pnp_ransac: offs[0] must be 0");
    if (nprob > 65535) return fail(ODO_ERR_CAPACITY, "pnp_ransac: more than 65535 problems per call");
    for (int p = 0; p < nprob; p++) {
        const int n = offs[p + 1] - offs[p];
        if (n < 0) return fail(ODO_ERR_ARG, "pnp_ransac: offsets must not decrease");
        if (n > pnp_ransac_max_points()) return fail(ODO_ERR_CAPACITY, "pnp_ransac: too many points");
    }
    const int total = offs[nprob];
    if ((size_t)H * (size_t)std::max(total, 1) > ((size_t)1 << 28))
        return fail(ODO_ERR_CAPACITY, "pnp_ransac: iterations x points");
    hipStream_t st = c->stream;
    DevArena& A = c->arena;
    A.begin();
    const size_t tn = (size_t)std::max(total, 1), P = (size_t)nprob;
    DevBuf dx(A, tn * 12), duv(A, tn * 8), doffs(A, (P + 1) * 4), didx(A, P * H * 5 * 4), dmodel(A, P * H * 6 * 8),
        dR(A, P * H * 9 * 8), dmask(A, (size_t)H * tn), dgood(A, P * H * 4), dstate(A, P * 4 * 4),
        dres(A, P * sizeof(odo_pnp_ransac_result)), dmo(A, tn);
    ARENA_CHECK(A);
    if (total) {
        HIPCHK(hipMemcpyAsync(dx.p, Xw, (size_t)total * 12, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(duv.p, uv, (size_t)total * 8, hipMemcpyHostToDevice, st));
    }
    HIPCHK(hipMemcpyAsync(doffs.p, offs, (P + 1) * 4, hipMemcpyHostToDevice, st));
    const odo_calib& k = calib ? *calib : c->cfg.calib;
    const float K4[4] = {k.fx, k.fy, k.cx, k.cy};
    launch_pnp_ransac(st, dx.as<float>(), duv.as<float>(), doffs.as<int>(), nprob, K4, H, reproj_err, confidence,
                      didx.as<int>(), dmodel.as<double>(), dR.as<double>(), dmask.as<uint8_t>(), dgood.as<int>(),
                      dstate.as<int>(), dres.as<odo_pnp_ransac_result>(), dmo.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(res, dres.p, P * sizeof(odo_pnp_ransac_result), hipMemcpyDeviceToHost, st));
    if (inlier_mask && total) HIPCHK(hipMemcpyAsync(inlier_mask, dmo.p, (size_t)total, hipMemcpyDeviceToHost, st));
    if (good_counts) HIPCHK(hipMemcpyAsync(good_counts, dgood.p, P * H * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return ODO_OK;
}

int odo_pnp_ransac(odo_ctx* c, const float* Xw, const float* uv, int n, const odo_calib* calib, int iterations,
                   float reproj_err, double confidence, odo_pnp_ransac_result* res, uint8_t* inlier_mask,
                   int32_t* good_counts) {
    if (!c || n < 0 || (n && (!Xw || !uv)) || !res) return fail(ODO_ERR_ARG, "bad pnp_ransac args");
    if (!(confidence > 0.0 && confidence < 1.0)) return fail(ODO_ERR_ARG, "confidence must be in (0, 1)");
    memset(res, 0, sizeof(*res));
    res->best_iter = -1;
    if (n < 10) {  // pnpransac.cpp:30: return 0 before solvePnPRansac
        if (inlier_mask && n) memset(inlier_mask, 0, (size_t)n);
        return ODO_OK;
    }
    const int32_t offs[2] = {0, n};
    return pnp_ransac_run(c, Xw, uv, offs, 1, calib, iterations, reproj_err, confidence, res, inlier_mask,
                          good_counts);
}

int odo_pnp_ransac_batch(odo_ctx* c, const float* Xw, const float* uv, const int32_t* offs, int nprob,
                         const odo_calib* calib, int iterations, float reproj_err, double confidence,
                         odo_pnp_ransac_result* res, uint8_t* inlier_mask) {
    if (!c || nprob < 0 || !offs || (nprob && !res)) return fail(ODO_ERR_ARG, "bad pnp_ransac_batch args");
    if (nprob == 0) return ODO_OK;
    if (offs[nprob] > 0 && (!Xw || !uv)) return fail(ODO_ERR_ARG, "bad pnp_ransac_batch args");
    return pnp_ransac_run(c, Xw, uv, offs, nprob, calib, iterations, reproj_err, confidence, res, inlier_mask,
                          nullptr);
}

static int gicp_run(odo_ctx* c, const float* src, const int32_t* soffs, const float* tgt, const int32_t* toffs,
                    const float* guesses, int nprob, int max_iterations, double max_corr_dist, float* T12,
                    int32_t* converged, int32_t* iterations, int32_t* n_corr) {
    if (soffs[0] != 0 || toffs[0] != 0) return fail(ODO_ERR_ARG, "gicp: offsets must start at 0");
    if (nprob > 65535) return fail(ODO_ERR_CAPACITY, "gicp: more than 65535 pairs per call");
    int max_ns = 0, max_nt = 0;
    for (int p = 0; p < nprob; p++) {
        const int ns = soffs[p + 1] - soffs[p], nt = toffs[p + 1] - toffs[p];
        if (ns < 0 || nt < 0) return fail(ODO_ERR_ARG, "gicp: offsets must not decrease");
        // brute-force neighbour searches: O(ns * nt) per ICP iteration in one workgroup
        if (ns > 16384 || nt > 16384) return fail(ODO_ERR_CAPACITY, "gicp: more than 16384 points in a cloud");
        max_ns = std::max(max_ns, ns);
        max_nt = std::max(max_nt, nt);
    }
    const size_t S = (size_t)std::max(soffs[nprob], 1), T = (size_t)std::max(toffs[nprob], 1), P = (size_t)nprob;
    hipStream_t st = c->stream;
    DevArena& A = c->arena;
    A.begin();
    DevBuf ds(A, S * 12), dt(A, T * 12), dCs(A, S * 72), dCt(A, T * 72), dout(A, S * 12), dM(A, S * 72), dis(A, S * 4),
        dit(A, S * 4), dT(A, P * 64), dio(A, P * 16), dg(A, P * 64), dso(A, (P + 1) * 4), dto(A, (P + 1) * 4);
    ARENA_CHECK(A);
    if (soffs[nprob]) HIPCHK(hipMemcpyAsync(ds.p, src, (size_t)soffs[nprob] * 12, hipMemcpyHostToDevice, st));
    if (toffs[nprob]) HIPCHK(hipMemcpyAsync(dt.p, tgt, (size_t)toffs[nprob] * 12, hipMemcpyHostToDevice, st));
    std::vector<float> g(16 * P);
    for (size_t p = 0; p < P; p++)
        for (int i = 0; i < 16; i++) g[16 * p + i] = guesses ? guesses[16 * p + i] : (i % 5 == 0 ? 1.f : 0.f);
    HIPCHK(hipMemcpyAsync(dg.p, g.data(), P * 64, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dso.p, soffs, (P + 1) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dto.p, toffs, (P + 1) * 4, hipMemcpyHostToDevice, st));
    GicpArgs args{dg.as<float>(), dso.as<int>(), dto.as<int>(), max_corr_dist, max_iterations, 20 /* PCL inner */};
    launch_gicp(st, ds.as<float>(), dt.as<float>(), nprob, max_ns, max_nt, dCs.as<double>(), dCt.as<double>(),
                dout.as<float>(), dM.as<double>(), dis.as<int>(), dit.as<int>(), args, dT.as<float>(), dio.as<int>());
    HIPCHK(hipGetLastError());
    std::vector<int> io(4 * P);
    HIPCHK(hipMemcpyAsync(T12, dT.p, P * 64, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(io.data(), dio.p, P * 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (size_t p = 0; p < P; p++) {
        converged[p] = io[4 * p];
        iterations[p] = io[4 * p + 1];
        n_corr[p] = io[4 * p + 2];
    }
    return ODO_OK;
}

int odo_gicp(odo_ctx* c, const float* src, int ns, const float* tgt, int nt, const float guess[16], int max_iterations,
             double max_corr_dist, float T12[16], int* converged, int* iterations, int* n_corr) {
    if (!c || ns < 0 || nt < 0 || (ns && !src) || (nt && !tgt) || !T12 || !converged || !iterations || !n_corr)
        return fail(ODO_ERR_ARG, "bad gicp args");
    *converged = 0;
    *iterations = 0;
    *n_corr = 0;
    for (int i = 0; i < 16; i++) T12[i] = i % 5 == 0 ? 1.f : 0.f;
    if (ns < 20 || nt < 20) return ODO_OK;  // generalizedicp.cpp:33
    const int32_t so[2] = {0, ns}, to[2] = {0, nt};
    return gicp_run(c, src, so, tgt, to, guess, 1, max_iterations, max_corr_dist, T12, converged, iterations, n_corr);
}

int odo_gicp_batch(odo_ctx* c, const float* src, const int32_t* soffs, const float* tgt, const int32_t* toffs,
                   const float* guesses, int nprob, int max_iterations, double max_corr_dist, float* T12,
                   int32_t* converged, int32_t* iterations, int32_t* n_corr) {
    if (!c || nprob < 0 || !soffs || !toffs || (nprob && (!T12 || !converged || !iterations || !n_corr)))
        return fail(ODO_ERR_ARG, "bad gicp_batch args");
    if (nprob == 0) return ODO_OK;
    if ((soffs[nprob] > 0 && !src) || (toffs[nprob] > 0 && !tgt)) return fail(ODO_ERR_ARG, "bad gicp_batch args");
    return gicp_run(c, src, soffs, tgt, toffs, guesses, nprob, max_iterations, max_corr_dist, T12, converged,
                    iterations, n_corr);
}

// Frame::ComputeImageBounds: cv::undistortPoints of the four corners (5
// iterations in double, App. A.10)
static void undistort_host(float u, float v, const odo_calib& c, float* uo, float* vo) {
    const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    const double k0 = c.k1, k1 = c.k2, k2 = c.p1, k3 = c.p2, k4 = c.k3;
    double x = u, y = v;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        double icdist = 1 / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
        double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x);
        double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    *uo = (float)(fx * x + cx);
    *vo = (float)(fy * y + cy);
}

int odo_image_bounds(odo_ctx* c, float b[4]) {
    if (!c || !b) return fail(ODO_ERR_ARG, "bad bounds args");
    const odo_calib& k = c->cfg.calib;
    if (k.k1 != 0.0f) {
        const float cu[4] = {0.f, (float)c->W, 0.f, (float)c->W}, cv_[4] = {0.f, 0.f, (float)c->H, (float)c->H};
        float u[4], v[4];
        for (int i = 0; i < 4; i++) undistort_host(cu[i], cv_[i], k, &u[i], &v[i]);
        b[0] = std::min(u[0], u[2]);
        b[1] = std::max(u[1], u[3]);
        b[2] = std::min(v[0], v[1]);
        b[3] = std::max(v[2], v[3]);
    } else {
        b[0] = 0.f;
        b[1] = (float)c->W;
        b[2] = 0.f;
        b[3] = (float)c->H;
    }
    return ODO_OK;
}

int odo_projection_match(odo_ctx* c, const float Tcw[16], const odo_landmark* lms, int nL, const float* kun,
                         const int32_t* octave, const uint8_t* desc, int n, const uint8_t* slot_taken, float th,
                         float nn_ratio, int32_t* slot_lm, float* proj, int* n_matches) {
    if (!c || !Tcw || nL < 0 || n < 0 || (nL && (!lms || !proj)) || (n && (!kun || !octave || !desc || !slot_lm)) ||
        !n_matches)
        return fail(ODO_ERR_ARG, "bad projection_match args");
    if (n > 8191) return fail(ODO_ERR_CAPACITY, "more than 8191 keypoints");
    *n_matches = 0;
    hipStream_t st = c->stream;
    float bounds[4];
    odo_image_bounds(c, bounds);
    const odo_calib& k = c->cfg.calib;
    const float cal5[5] = {k.fx, k.fy, k.cx, k.cy, k.mbf};
    const size_t nl = std::max(nL, 1), nn = std::max(n, 1);
    DevArena& A = c->arena;
    A.begin();
    DevBuf dT(A, 64), dl(A, nl * sizeof(odo_landmark)), dk(A, nn * 8), doc(A, nn * 4), dd(A, nn * 32), dtk(A, nn),
        dproj(A, nl * 12), din(A, nl), dcc(A, nl * 4), dcand(A, nl * projection_cand_cap() * 4), dsl(A, nn * 4),
        dnm(A, 4);
    ARENA_CHECK(A);
    HIPCHK(hipMemcpyAsync(dT.p, Tcw, 64, hipMemcpyHostToDevice, st));
    if (nL) HIPCHK(hipMemcpyAsync(dl.p, lms, (size_t)nL * sizeof(odo_landmark), hipMemcpyHostToDevice, st));
    if (n) {
        HIPCHK(hipMemcpyAsync(dk.p, kun, (size_t)n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(doc.p, octave, (size_t)n * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(dd.p, desc, (size_t)n * 32, hipMemcpyHostToDevice, st));
        if (slot_taken) HIPCHK(hipMemcpyAsync(dtk.p, slot_taken, (size_t)n, hipMemcpyHostToDevice, st));
        else HIPCHK(hipMemsetAsync(dtk.p, 0, (size_t)n, st));
    }
    if (launch_projection_match(st, dT.as<float>(), dl.as<odo_landmark>(), nL, dk.as<float>(), doc.as<int32_t>(),
                                dd.as<uint8_t>(), n, dtk.as<uint8_t>(), cal5, bounds, th, nn_ratio, dproj.as<float>(),
                                din.as<uint8_t>(), dcc.as<int>(), dcand.as<uint32_t>(), dsl.as<int32_t>(),
                                dnm.as<int>()) != 0)
        return fail(ODO_ERR_CAPACITY, "projection match capacity");
    HIPCHK(hipGetLastError());
    if (nL) HIPCHK(hipMemcpyAsync(proj, dproj.p, (size_t)nL * 12, hipMemcpyDeviceToHost, st));
    if (n) HIPCHK(hipMemcpyAsync(slot_lm, dsl.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(n_matches, dnm.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return ODO_OK;
}

int odo_chain_poses(const odo_pair_result* res, int n, const float Tcw_prev[16], float* out) {
    if (!res || n < 0 || !out) return fail(ODO_ERR_ARG, "bad chain args");
    double T[16];
    for (int k = 0; k < 16; k++) T[k] = Tcw_prev ? (double)Tcw_prev[k] : (k % 5 == 0 ? 1.0 : 0.0);
    for (int i = 0; i < n; i++) {
        if (!(i == 0 && res[i].n_matches == 0)) {
            double R[16], M[16];
            for (int k = 0; k < 16; k++) R[k] = (double)res[i].Tcw[k];
            for (int r = 0; r < 4; r++)
                for (int c2 = 0; c2 < 4; c2++)
                    M[4 * r + c2] = ((R[4 * r] * T[c2] + R[4 * r + 1] * T[4 + c2]) + R[4 * r + 2] * T[8 + c2]) +
                                    R[4 * r + 3] * T[12 + c2];
            memcpy(T, M, sizeof(T));
        }
        for (int k = 0; k < 16; k++) out[16 * i + k] = (float)T[k];
    }
    return ODO_OK;
}

// Eigen::Quaterniond(Matrix3d) (quaternionbase_assign_impl), host restatement
static void quat_from_rot(const double m[3][3], double q[4] /* x y z w */) {
    double t = m[0][0] + m[1][1] + m[2][2];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[2][1] - m[1][2]) * t;
        q[1] = (m[0][2] - m[2][0]) * t;
        q[2] = (m[1][0] - m[0][1]) * t;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > m[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[k][j] - m[j][k]) * t;
        q[j] = (m[j][i] + m[i][j]) * t;
        q[k] = (m[k][i] + m[i][k]) * t;
    }
}

int odo_write_tum_trajectory(const char* path, const double* ts, const float* Tcw, int n, int append) {
    if (!path || n < 0 || (n && (!ts || !Tcw))) return fail(ODO_ERR_ARG, "bad trajectory args");
    FILE* f = fopen(path, append ? "a" : "w");
    if (!f) return fail(ODO_ERR_ARG, std::string("cannot open ") + path);
    for (int i = 0; i < n; i++) {
        const float* T = Tcw + 16 * i;
        // Rwc = Rcw^T; twc = -Rwc * tcw (cv::Mat float, double accumulation)
        float Rwc[3][3];
        for (int r = 0; r < 3; r++)
            for (int c2 = 0; c2 < 3; c2++) Rwc[r][c2] = T[4 * c2 + r];
        float twc[3];
        for (int r = 0; r < 3; r++)
            twc[r] = (float)(((double)-Rwc[r][0] * T[3] + (double)-Rwc[r][1] * T[7]) + (double)-Rwc[r][2] * T[11]);
        double m[3][3], q[4];
        for (int r = 0; r < 3; r++)
            for (int c2 = 0; c2 < 3; c2++) m[r][c2] = (double)Rwc[r][c2];
        quat_from_rot(m, q);
        fprintf(f, "%.6f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", ts[i], twc[0], twc[1], twc[2], (float)q[0],
                (float)q[1], (float)q[2], (float)q[3]);
    }
    fclose(f);
    return ODO_OK;
}

int odo_kabsch(const float* A, const float* B, int n, float T[16]) {
    if (n < 0 || (n && (!A || !B)) || !T) return fail(ODO_ERR_ARG, "bad kabsch args");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(ODO_ERR_DEVICE, "no HIP device");
    const int kc = std::max(n, 1);
    // Kabsch::Compute takes no context: one process-wide arena, one caller at a time
    static std::mutex mu;
    static DevArena KA;
    std::lock_guard<std::mutex> lock(mu);
    KA.begin();
    DevBuf da(KA, (size_t)kc * 12), db(KA, (size_t)kc * 12), dT(KA, 64);
    ARENA_CHECK(KA);
    if (n) {
        HIPCHK(hipMemcpy(da.p, A, (size_t)n * 12, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(db.p, B, (size_t)n * 12, hipMemcpyHostToDevice));
    }
    launch_kabsch(0, da.as<float>(), db.as<float>(), n, dT.as<float>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(T, dT.p, 64, hipMemcpyDeviceToHost));
    return ODO_OK;
}

}  // extern "C"
