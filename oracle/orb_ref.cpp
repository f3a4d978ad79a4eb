// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of the
// ORB-SLAM2 extractor used on the reference's hot path:
//   Frame::Frame            Core/frame.cpp:18-45
//   ORBextractor ctor       Features/orbextractor.cpp:346-404
//   ComputePyramid          Features/orbextractor.cpp:833-857
//   ComputeKeyPointsOctTree Features/orbextractor.cpp:665-746
//   DistributeOctTree       Features/orbextractor.cpp:466-663
//   IC_Angle                Features/orbextractor.cpp:14-39
//   computeOrbDescriptor    Features/orbextractor.cpp:43-85
//   operator()              Features/orbextractor.cpp:756-815
// OpenCV internals (cvtColor, resize, FAST, GaussianBlur, fastAtan2, cvRound)
// follow SURVEY.md Appendix A; choices the survey left open are recorded in
// DESIGN.md §4 ("pinned choices").
#include <cfloat>
#include <cmath>
#include <cstring>
#include <list>
#include <vector>
#include <algorithm>
#include <utility>

#include "oracle.h"
#include "../include/odo_orb_pattern.h"

namespace {

const int PATCH_SIZE = 31;
const int HALF_PATCH_SIZE = 15;
const int EDGE_THRESHOLD = 19;

inline int cvRound(float v) { return (int)lrintf(v); }   // round half to even
inline int cvRound(double v) { return (int)lrint(v); }
inline int cvFloor(float v) { int i = (int)v; return i - (i > v); }
inline int cvFloor(double v) { int i = (int)v; return i - (i > v); }
inline int cvCeil(float v) { int i = (int)v; return i + (i < v); }
inline short sat_short(float v) {
    int r = cvRound(v);
    return (short)std::min(std::max(r, -32768), 32767);
}

struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
};

struct KP {
    float x, y, size, angle, response;
    int octave, class_id;
};

// ---------------------------------------------------------------- A.1
void bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray) {
    for (int y = 0; y < h; ++y) {
        const uint8_t* row = bgr + (size_t)y * stride;
        for (int x = 0; x < w; ++x) {
            int b = row[3 * x], g = row[3 * x + 1], r = row[3 * x + 2];
            gray[(size_t)y * w + x] = (uint8_t)((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14);
        }
    }
}

// ---------------------------------------------------------------- tables
struct Tables {
    int nlevels, nfeatures;
    std::vector<float> scale, inv_scale, sigma2;
    std::vector<int> quota;
    std::vector<int> umax;
};

Tables make_tables(const odo_orb_params& p) {
    // orbextractor.cpp:346-404. scaleFactor member is double (orbextractor.h)
    Tables t;
    t.nlevels = p.nlevels;
    t.nfeatures = p.nfeatures;
    const double scaleFactor = (double)p.scale_factor;
    t.scale.resize(p.nlevels);
    t.sigma2.resize(p.nlevels);
    t.scale[0] = 1.0f;
    t.sigma2[0] = 1.0f;
    for (int i = 1; i < p.nlevels; i++) {
        t.scale[i] = (float)((double)t.scale[i - 1] * scaleFactor);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    t.inv_scale.resize(p.nlevels);
    for (int i = 0; i < p.nlevels; i++) t.inv_scale[i] = 1.0f / t.scale[i];

    t.quota.resize(p.nlevels);
    float factor = (float)(1.0f / scaleFactor);
    float nDesired = p.nfeatures * (1 - factor) / (1 - (float)pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int level = 0; level < p.nlevels - 1; level++) {
        t.quota[level] = cvRound(nDesired);
        sum += t.quota[level];
        nDesired *= factor;
    }
    t.quota[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);

    t.umax.resize(HALF_PATCH_SIZE + 1);
    int v, v0, vmax = cvFloor(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    int vmin = cvCeil(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) t.umax[v] = cvRound(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    return t;
}

// ---------------------------------------------------------------- A.2
// cv::resize(INTER_LINEAR) for 8U, generic fixed-point path; vertical pass
// uses the scalar formula everywhere (App. A.2).
void resize_linear(const Img& src, Img& dst, int dw, int dh) {
    dst.w = dw;
    dst.h = dh;
    dst.px.assign((size_t)dw * dh, 0);
    const double inv_scale_x = (double)dw / src.w, inv_scale_y = (double)dh / src.h;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    std::vector<int> xofs(dw);
    std::vector<short> alpha(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cvFloor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= src.w) {
            xmax = std::min(xmax, dx);
            if (sx >= src.w - 1) { fx = 0; sx = src.w - 1; }
        }
        xofs[dx] = sx;
        alpha[2 * dx] = sat_short((1.f - fx) * 2048);
        alpha[2 * dx + 1] = sat_short(fx * 2048);
    }
    std::vector<int> row0(dw), row1(dw);
    auto hresize = [&](int sy, std::vector<int>& out) {
        const uint8_t* S = &src.px[(size_t)sy * src.w];
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) out[dx] = S[sx] * alpha[2 * dx] + S[sx + 1] * alpha[2 * dx + 1];
            else out[dx] = S[sx] * 2048;
        }
    };
    auto clip = [&](int y) { return y < 0 ? 0 : (y >= src.h ? src.h - 1 : y); };
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cvFloor(fy);
        fy -= sy;
        int b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
        hresize(clip(sy), row0);
        hresize(clip(sy + 1), row1);
        for (int dx = 0; dx < dw; dx++) {
            int v = (row0[dx] * b0 + row1[dx] * b1 + (1 << 21)) >> 22;
            dst.px[(size_t)dy * dw + dx] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
}

// ---------------------------------------------------------------- A.3 FAST
const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

// cornerScore<16> (opencv fast_score.cpp), restated.
int corner_score(const uint8_t* ptr, const int* pixel, int threshold) {
    const int K = 8, N = K * 3 + 1;
    int v = ptr[0];
    short d[N];
    for (int k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min((int)d[k + 1], (int)d[k + 2]);
        a = std::min(a, (int)d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, (int)d[k + 4]);
        a = std::min(a, (int)d[k + 5]);
        a = std::min(a, (int)d[k + 6]);
        a = std::min(a, (int)d[k + 7]);
        a = std::min(a, (int)d[k + 8]);
        a0 = std::max(a0, std::min(a, (int)d[k]));
        a0 = std::max(a0, std::min(a, (int)d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max((int)d[k + 1], (int)d[k + 2]);
        b = std::max(b, (int)d[k + 3]);
        b = std::max(b, (int)d[k + 4]);
        b = std::max(b, (int)d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, (int)d[k + 6]);
        b = std::max(b, (int)d[k + 7]);
        b = std::max(b, (int)d[k + 8]);
        b0 = std::min(b0, std::max(b, (int)d[k]));
        b0 = std::min(b0, std::max(b, (int)d[k + 9]));
    }
    return -b0 - 1;
}

// cv::FAST(roi, kps, threshold, nonmax=true) TYPE_9_16 on an ROI given by
// base pointer / stride / size: FAST_t<16> restated (scores stored as uchar,
// NMS strictly greater than the 8 neighbours, row-major emission).
void fast_roi(const uint8_t* base, int stride, int rows, int cols, int threshold,
              std::vector<KP>& out) {
    out.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    int pixel[25];
    for (int k = 0; k < 16; k++) pixel[k] = kCircle[k][0] + kCircle[k][1] * stride;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
    std::vector<uint8_t> score((size_t)rows * cols, 0);
    std::vector<uint8_t> is_corner((size_t)rows * cols, 0);
    for (int i = 3; i < rows - 3; i++) {
        for (int j = 3; j < cols - 3; j++) {
            const uint8_t* ptr = base + (size_t)i * stride + j;
            int v = ptr[0];
            // darker run
            bool corner = false;
            {
                int vt = v - threshold, count = 0;
                for (int k = 0; k < 25; k++) {
                    int x = ptr[pixel[k]];
                    if (x < vt) {
                        if (++count > 8) { corner = true; break; }
                    } else count = 0;
                }
            }
            if (!corner) {
                int vt = v + threshold, count = 0;
                for (int k = 0; k < 25; k++) {
                    int x = ptr[pixel[k]];
                    if (x > vt) {
                        if (++count > 8) { corner = true; break; }
                    } else count = 0;
                }
            }
            if (corner) {
                is_corner[(size_t)i * cols + j] = 1;
                score[(size_t)i * cols + j] = (uint8_t)corner_score(ptr, pixel, threshold);
            }
        }
    }
    for (int i = 3; i < rows - 3; i++) {
        for (int j = 3; j < cols - 3; j++) {
            if (!is_corner[(size_t)i * cols + j]) continue;
            int s = score[(size_t)i * cols + j];
            bool keep = true;
            for (int di = -1; di <= 1 && keep; di++)
                for (int dj = -1; dj <= 1; dj++) {
                    if (!di && !dj) continue;
                    if (!(s > score[(size_t)(i + di) * cols + (j + dj)])) { keep = false; break; }
                }
            if (keep) out.push_back(KP{(float)j, (float)i, 7.f, -1.f, (float)s, 0, -1});
        }
    }
}

// ComputeKeyPointsOctTree FAST part (orbextractor.cpp:669-723).
void fast_level(const Img& im, int iniTh, int minTh, std::vector<KP>& cands) {
    const float W = 30;
    const int minBorderX = EDGE_THRESHOLD - 3;
    const int minBorderY = minBorderX;
    const int maxBorderX = im.w - EDGE_THRESHOLD + 3;
    const int maxBorderY = im.h - EDGE_THRESHOLD + 3;
    cands.clear();
    const float width = (maxBorderX - minBorderX);
    const float height = (maxBorderY - minBorderY);
    const int nCols = width / W;
    const int nRows = height / W;
    const int wCell = ceil(width / nCols);
    const int hCell = ceil(height / nRows);
    std::vector<KP> cell;
    for (int i = 0; i < nRows; i++) {
        const float iniY = minBorderY + i * hCell;
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBorderY - 3) continue;
        if (maxY > maxBorderY) maxY = maxBorderY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = minBorderX + j * wCell;
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = maxBorderX;
            const int y0 = (int)iniY, y1 = (int)maxY, x0 = (int)iniX, x1 = (int)maxX;
            const uint8_t* base = &im.px[(size_t)y0 * im.w + x0];
            fast_roi(base, im.w, y1 - y0, x1 - x0, iniTh, cell);
            if (cell.empty()) fast_roi(base, im.w, y1 - y0, x1 - x0, minTh, cell);
            for (auto& k : cell) {
                k.x += j * wCell;
                k.y += i * hCell;
                cands.push_back(k);
            }
        }
    }
}

// ---------------------------------------------------------------- octree
struct Pt2i { int x, y; };
struct Node {
    std::vector<KP> vKeys;
    Pt2i UL, UR, BL, BR;
    std::list<Node>::iterator lit;
    bool bNoMore = false;
    long long seq = 0;  // creation order: pinned tie-break for (size, pointer) sort
};

void divide_node(const Node& n, Node& n1, Node& n2, Node& n3, Node& n4) {
    const int halfX = ceil(static_cast<float>(n.UR.x - n.UL.x) / 2);
    const int halfY = ceil(static_cast<float>(n.BR.y - n.UL.y) / 2);
    n1.UL = n.UL;
    n1.UR = Pt2i{n.UL.x + halfX, n.UL.y};
    n1.BL = Pt2i{n.UL.x, n.UL.y + halfY};
    n1.BR = Pt2i{n.UL.x + halfX, n.UL.y + halfY};
    n2.UL = n1.UR;
    n2.UR = n.UR;
    n2.BL = n1.BR;
    n2.BR = Pt2i{n.UR.x, n.UL.y + halfY};
    n3.UL = n1.BL;
    n3.UR = n1.BR;
    n3.BL = n.BL;
    n3.BR = Pt2i{n1.BR.x, n.BL.y};
    n4.UL = n3.UR;
    n4.UR = n2.BR;
    n4.BL = n3.BR;
    n4.BR = n.BR;
    for (const KP& kp : n.vKeys) {
        if (kp.x < n1.UR.x) {
            if (kp.y < n1.BR.y) n1.vKeys.push_back(kp);
            else n3.vKeys.push_back(kp);
        } else if (kp.y < n1.BR.y) n2.vKeys.push_back(kp);
        else n4.vKeys.push_back(kp);
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

struct SizePtr {
    int size;
    Node* node;
    bool operator<(const SizePtr& o) const {
        if (size != o.size) return size < o.size;
        return node->seq < o.node->seq;
    }
};

std::vector<KP> distribute_octree(const std::vector<KP>& keys, int minX, int maxX, int minY,
                                  int maxY, int N) {
    const int nIni = round(static_cast<float>(maxX - minX) / (maxY - minY));
    const float hX = static_cast<float>(maxX - minX) / nIni;
    std::list<Node> lNodes;
    std::vector<Node*> ini(nIni);
    long long seq = 0;
    for (int i = 0; i < nIni; i++) {
        Node ni;
        ni.UL = Pt2i{(int)(hX * static_cast<float>(i)), 0};
        ni.UR = Pt2i{(int)(hX * static_cast<float>(i + 1)), 0};
        ni.BL = Pt2i{ni.UL.x, maxY - minY};
        ni.BR = Pt2i{ni.UR.x, maxY - minY};
        ni.seq = seq++;
        lNodes.push_back(ni);
        ini[i] = &lNodes.back();
    }
    for (const KP& kp : keys) ini[(size_t)(kp.x / hX)]->vKeys.push_back(kp);

    auto lit = lNodes.begin();
    while (lit != lNodes.end()) {
        if (lit->vKeys.size() == 1) {
            lit->bNoMore = true;
            lit++;
        } else if (lit->vKeys.empty()) lit = lNodes.erase(lit);
        else lit++;
    }

    bool bFinish = false;
    std::vector<SizePtr> vSizeAndPtr;
    auto push_child = [&](Node& c, std::vector<SizePtr>& acc, int* nToExpand) {
        if (c.vKeys.size() > 0) {
            c.seq = seq++;
            lNodes.push_front(c);
            if (c.vKeys.size() > 1) {
                if (nToExpand) (*nToExpand)++;
                acc.push_back(SizePtr{(int)c.vKeys.size(), &lNodes.front()});
                lNodes.front().lit = lNodes.begin();
            }
        }
    };
    while (!bFinish) {
        int prevSize = lNodes.size();
        lit = lNodes.begin();
        int nToExpand = 0;
        vSizeAndPtr.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) {
                lit++;
                continue;
            }
            Node n1, n2, n3, n4;
            divide_node(*lit, n1, n2, n3, n4);
            push_child(n1, vSizeAndPtr, &nToExpand);
            push_child(n2, vSizeAndPtr, &nToExpand);
            push_child(n3, vSizeAndPtr, &nToExpand);
            push_child(n4, vSizeAndPtr, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if (((int)lNodes.size() + nToExpand * 3) > N) {
            while (!bFinish) {
                prevSize = lNodes.size();
                std::vector<SizePtr> vPrev = vSizeAndPtr;
                vSizeAndPtr.clear();
                std::sort(vPrev.begin(), vPrev.end());
                for (int j = (int)vPrev.size() - 1; j >= 0; j--) {
                    Node n1, n2, n3, n4;
                    divide_node(*vPrev[j].node, n1, n2, n3, n4);
                    push_child(n1, vSizeAndPtr, nullptr);
                    push_child(n2, vSizeAndPtr, nullptr);
                    push_child(n3, vSizeAndPtr, nullptr);
                    push_child(n4, vSizeAndPtr, nullptr);
                    lNodes.erase(vPrev[j].node->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<KP> res;
    res.reserve(lNodes.size());
    for (auto& n : lNodes) {
        const KP* best = &n.vKeys[0];
        float maxResponse = best->response;
        for (size_t k = 1; k < n.vKeys.size(); k++)
            if (n.vKeys[k].response > maxResponse) {
                best = &n.vKeys[k];
                maxResponse = n.vKeys[k].response;
            }
        res.push_back(*best);
    }
    return res;
}

// ---------------------------------------------------------------- A.5
float fast_atan2(float y, float x) {
    static const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    static const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    static const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    static const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = std::abs(x), ay = std::abs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

float ic_angle(const Img& im, float px, float py, const std::vector<int>& umax) {
    int m_01 = 0, m_10 = 0;
    const int cy = cvRound(py), cx = cvRound(px);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * im.at(cy, cx + u);
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = im.at(cy + v, cx + u), val_minus = im.at(cy - v, cx + u);
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// ---------------------------------------------------------------- A.4
const int kGauss[7] = {18, 34, 48, 56, 48, 34, 18};  // Q8, error-diffused, sum 256

inline int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        else i = 2 * n - 2 - i;
    }
    return i;
}

void gaussian_blur(const Img& src, Img& dst) {
    dst.w = src.w;
    dst.h = src.h;
    dst.px.assign(src.px.size(), 0);
    std::vector<uint32_t> H((size_t)src.w * src.h);
    for (int y = 0; y < src.h; y++)
        for (int x = 0; x < src.w; x++) {
            uint32_t s = 0;
            for (int j = -3; j <= 3; j++) s += kGauss[j + 3] * src.at(y, reflect101(x + j, src.w));
            H[(size_t)y * src.w + x] = s;
        }
    for (int y = 0; y < src.h; y++)
        for (int x = 0; x < src.w; x++) {
            uint32_t s = 0;
            for (int j = -3; j <= 3; j++) s += kGauss[j + 3] * H[(size_t)reflect101(y + j, src.h) * src.w + x];
            dst.px[(size_t)y * src.w + x] = (uint8_t)((s + 32768) >> 16);
        }
}

// computeOrbDescriptor (orbextractor.cpp:43-85); cos/sin of the float angle
// are taken in double and rounded to float (App. A.5 note).
void orb_descriptor(const KP& kpt, const Img& img, uint8_t* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    float angle = (float)kpt.angle * factorPI;
    float a = (float)cos((double)angle), b = (float)sin((double)angle);
    const int cy = cvRound(kpt.y), cx = cvRound(kpt.x);
    const int8_t* pattern = ODO_ORB_PATTERN;
    auto value = [&](int idx) {
        float px = (float)pattern[2 * idx], py = (float)pattern[2 * idx + 1];
        int yy = cvRound(px * b + py * a);
        int xx = cvRound(px * a - py * b);
        return (int)img.at(cy + yy, cx + xx);
    };
    for (int i = 0; i < 32; ++i, pattern += 32) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            int t0 = value(2 * bit), t1 = value(2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

// ---------------------------------------------------------------- extractor
struct Extractor {
    Tables t;
    std::vector<Img> pyr;
    explicit Extractor(const odo_orb_params& p) : t(make_tables(p)) {}

    void compute_pyramid(const uint8_t* gray, int w, int h) {
        pyr.assign(t.nlevels, Img());
        for (int level = 0; level < t.nlevels; ++level) {
            float s = t.inv_scale[level];
            int sw = cvRound((float)w * s), sh = cvRound((float)h * s);
            if (level == 0) {
                pyr[0].w = w;
                pyr[0].h = h;
                pyr[0].px.assign(gray, gray + (size_t)w * h);
            } else {
                resize_linear(pyr[level - 1], pyr[level], sw, sh);
            }
        }
    }

    int run(const uint8_t* gray, int w, int h, std::vector<KP>& out, std::vector<uint8_t>& desc) {
        out.clear();
        desc.clear();
        if (w <= 0 || h <= 0) return 0;
        compute_pyramid(gray, w, h);
        std::vector<std::vector<KP>> all(t.nlevels);
        for (int level = 0; level < t.nlevels; ++level) {
            const Img& im = pyr[level];
            const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
            const int maxBorderX = im.w - EDGE_THRESHOLD + 3, maxBorderY = im.h - EDGE_THRESHOLD + 3;
            std::vector<KP> cands;
            fast_level(im, ini_th, min_th, cands);
            if (!cands.empty())
                all[level] = distribute_octree(cands, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                               t.quota[level]);
            const int scaledPatchSize = PATCH_SIZE * t.scale[level];
            for (KP& k : all[level]) {
                k.x += minBorderX;
                k.y += minBorderY;
                k.octave = level;
                k.size = scaledPatchSize;
            }
        }
        for (int level = 0; level < t.nlevels; ++level)
            for (KP& k : all[level]) k.angle = ic_angle(pyr[level], k.x, k.y, t.umax);
        int total = 0;
        for (auto& v : all) total += (int)v.size();
        desc.assign((size_t)total * 32, 0);
        int offset = 0;
        for (int level = 0; level < t.nlevels; ++level) {
            std::vector<KP>& kps = all[level];
            if (kps.empty()) continue;
            Img blurred;
            gaussian_blur(pyr[level], blurred);
            for (size_t i = 0; i < kps.size(); i++) orb_descriptor(kps[i], blurred, &desc[(offset + i) * 32]);
            offset += (int)kps.size();
            if (level != 0) {
                float scale = t.scale[level];
                for (KP& k : kps) {
                    k.x *= scale;
                    k.y *= scale;
                }
            }
            out.insert(out.end(), kps.begin(), kps.end());
        }
        return total;
    }

    int ini_th = 20, min_th = 7;
};


// ---------------------------------------------------------------- ADAPTIVE
// Extractor(FAST, ORB, ADAPTIVE) (extractor.cpp:14-77): a 3x3
// VideoGridAdaptedFeatureDetector over VideoDynamicAdaptedFeatureDetector
// cells, each owning a DetectorAdjuster(FAST, 20, 2, 10000, 1.3, 0.7) whose
// threshold persists across frames; then KeyPointsFilter::retainBest and
// cv::ORB::compute. The libstdc++ selection algorithms are the real ones.

// keepStrongest / ResponseComparator (videogridadaptedfeaturedetector.cpp:17-31)
void keep_strongest(int N, std::vector<KP>& kps) {
    if ((int)kps.size() > N) {
        std::nth_element(kps.begin(), kps.begin() + N, kps.end(),
                         [](const KP& a, const KP& b) { return std::abs(a.response) > std::abs(b.response); });
        kps.erase(kps.begin() + N, kps.end());
    }
}

// cv::KeyPointsFilter::retainBest (OpenCV 3.4 keypoint.cpp): nth_element by
// response (greater), then partition the tail keeping the boundary ties.
void retain_best(std::vector<KP>& kps, int n_points) {
    if (n_points >= 0 && kps.size() > (size_t)n_points) {
        if (n_points == 0) {
            kps.clear();
            return;
        }
        std::nth_element(kps.begin(), kps.begin() + n_points, kps.end(),
                         [](const KP& a, const KP& b) { return a.response > b.response; });
        const float amb = kps[n_points - 1].response;
        auto new_end = std::partition(kps.begin() + n_points, kps.end(),
                                      [amb](const KP& k) { return k.response >= amb; });
        kps.resize(new_end - kps.begin());
    }
}

// One grid cell's stateful detector: VideoDynamicAdaptedFeatureDetector::detect
// (videodynamicadaptedfeaturedetector.cpp:24-44) over DetectorAdjuster
// (detectoradjuster.cpp:22-65) with the FAST inner detector: the double
// threshold is passed to FastFeatureDetector::create(int) (truncation).
int adaptive_cell_detect(const uint8_t* base, int stride, int rows, int cols, const odo_adaptive_params& p,
                         double& thresh, std::vector<KP>& kps) {
    int iterCount = p.escape_iters;
    int t_used = 0;
    do {
        kps.clear();
        t_used = (int)thresh;
        fast_roi(base, stride, rows, cols, t_used, kps);
        const int found = (int)kps.size();
        if (found < p.cell_min) {
            thresh *= p.decrease_factor;  // tooFew
            if (thresh < p.min_thresh) thresh = p.min_thresh;
        } else if (found > p.cell_max) {
            thresh *= p.increase_factor;  // tooMany
            if (thresh > p.max_thresh) thresh = p.max_thresh;
            break;
        } else
            break;
        iterCount--;
    } while (iterCount > 0 && (thresh > p.min_thresh) && (thresh < p.max_thresh));
    return std::min(std::max(t_used, 0), 255);
}

// VideoGridAdaptedFeatureDetector::detect (videogridadaptedfeaturedetector.cpp:52-84)
void adaptive_grid_detect(const uint8_t* gray, int w, int h, const odo_adaptive_params& p, double* thresh,
                          std::vector<KP>& out, int* t_used) {
    const int R = p.grid_rows, C = p.grid_cols, E = p.edge_threshold;
    const int maxPerCell = p.max_total_keypoints / (R * C);
    std::vector<std::vector<KP>> sub(R * C);
    for (int i = 0; i < R; ++i) {
        const int rs = std::max((i * h) / R - E, 0), re = std::min(h, ((i + 1) * h) / R + E);
        for (int j = 0; j < C; ++j) {
            const int cs = std::max((j * w) / C - E, 0), ce = std::min(w, ((j + 1) * w) / C + E);
            const int t = adaptive_cell_detect(gray + (size_t)rs * w + cs, w, re - rs, ce - cs, p, thresh[j + i * C],
                                               sub[j + i * C]);
            if (t_used) t_used[j + i * C] = t;
            keep_strongest(maxPerCell, sub[j + i * C]);
        }
    }
    out.clear();
    for (int i = 0; i < R; ++i) {  // aggregateKeypointsPerGridCell (:33-50)
        const int rs = std::max((i * h) / R - E, 0);
        for (int j = 0; j < C; ++j) {
            const int cs = std::max((j * w) / C - E, 0);
            for (KP& k : sub[j + i * C]) {
                k.x += cs;
                k.y += rs;
            }
            out.insert(out.end(), sub[j + i * C].begin(), sub[j + i * C].end());
        }
    }
}

// cv::ORB::compute on provided keypoints (OpenCV 3.4 orb.cpp detectAndCompute,
// useProvidedKeypoints): runByImageBorder(edgeThreshold 31), one pyramid level
// (every FAST keypoint has octave 0), GaussianBlur 7x7 sigma 2 REFLECT_101 of
// that level, rBRIEF at the keypoint's own angle (-1 for FAST keypoints: ORB
// does not orient provided keypoints).
void orb_compute_provided(const uint8_t* gray, int w, int h, std::vector<KP>& kps, std::vector<uint8_t>& desc) {
    const int border = 31;
    if (h <= 2 * border || w <= 2 * border) kps.clear();
    else {
        const float x0 = border, y0 = border, x1 = (float)(w - border), y1 = (float)(h - border);
        kps.erase(std::remove_if(kps.begin(), kps.end(),
                                 [&](const KP& k) { return !(x0 <= k.x && k.x < x1 && y0 <= k.y && k.y < y1); }),
                  kps.end());
    }
    desc.assign(kps.size() * 32, 0);
    if (kps.empty()) return;
    Img im, blurred;
    im.w = w;
    im.h = h;
    im.px.assign(gray, gray + (size_t)w * h);
    gaussian_blur(im, blurred);
    for (size_t i = 0; i < kps.size(); i++) orb_descriptor(kps[i], blurred, &desc[i * 32]);
}

int adaptive_extract(const uint8_t* gray, int w, int h, const odo_adaptive_params& p, double* thresh,
                     std::vector<KP>& kps, std::vector<uint8_t>& desc, int* t_used) {
    adaptive_grid_detect(gray, w, h, p, thresh, kps, t_used);
    if ((int)kps.size() > p.retain_best) retain_best(kps, p.retain_best);  // extractor.cpp:45-46
    orb_compute_provided(gray, w, h, kps, desc);
    return (int)kps.size();
}

// ---------------------------------------------------------------- ADAPTIVE, cv::ORB inner
// Extractor(ORB, ORB, ADAPTIVE) (extractor.cpp:52-77 with the ORB adjuster
// DetectorAdjuster(ORB, 20, 2, 10000, 1.3, 0.7)): every cell's detect() is
// cv::ORB::create(10000, 1.2f, 8, 15, 0, 2, HARRIS_SCORE, 31, (int)mThresh)
// ->detect(sub_image) (detectoradjuster.cpp:29), restated from OpenCV 3.4
// orb.cpp (detectAndCompute with do_keypoints, computeKeyPoints,
// HarrisResponses, ICAngles). Pinned choices (DESIGN.md §4 "ADAPTIVE, cv::ORB
// inner"): the pyramid uses the INTER_LINEAR resize of App. A.2 (OpenCV
// 3.4.0/3.4.1; later 3.4.x switched orb.cpp to INTER_LINEAR_EXACT).
const int OCV_NFEATURES = 10000, OCV_NLEVELS = 8, OCV_EDGE = 15, OCV_PATCH = 31, OCV_HARRIS_BLOCK = 7;
const float OCV_SCALE_FACTOR = 1.2f, OCV_HARRIS_K = 0.04f;

// ORB_Impl::getScale: (float)pow(scaleFactor, level) with the double member
// scaleFactor = (double)1.2f (not the cumulative float product of ORB-SLAM2).
float orbcv_scale(int level) { return (float)std::pow((double)OCV_SCALE_FACTOR, (double)level); }

// computeKeyPoints: nfeaturesPerLevel (geometric, cvRound, last = remainder)
std::vector<int> orbcv_quotas(int nfeatures, int nlevels) {
    std::vector<int> q(nlevels);
    const float factor = (float)(1.0 / (double)OCV_SCALE_FACTOR);
    float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        q[l] = cvRound(nd);
        sum += q[l];
        nd *= factor;
    }
    q[nlevels - 1] = std::max(nfeatures - sum, 0);
    return q;
}

// KeyPointsFilter::runByImageBorder (keypoint.cpp): keep Rect(b, b, w-2b, h-2b)
// .contains(pt) in order; everything goes when the image is too small.
void run_by_image_border(std::vector<KP>& kps, int w, int h, int b) {
    if (b <= 0) return;
    if (h <= 2 * b || w <= 2 * b) {
        kps.clear();
        return;
    }
    const float x0 = (float)b, y0 = (float)b, x1 = (float)(w - b), y1 = (float)(h - b);
    kps.erase(std::remove_if(kps.begin(), kps.end(),
                             [&](const KP& k) { return !(x0 <= k.x && k.x < x1 && y0 <= k.y && k.y < y1); }),
              kps.end());
}

// HarrisResponses (orb.cpp): 7x7 block of Sobel-like gradients around
// (cvRound(x), cvRound(y)) of the level, integer sums, float response.
float harris_response(const Img& im, int x0, int y0) {
    const int r = OCV_HARRIS_BLOCK / 2;
    const float scale = 1.f / ((1 << 2) * OCV_HARRIS_BLOCK * 255.f);
    const float scale_sq_sq = scale * scale * scale * scale;
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < OCV_HARRIS_BLOCK; i++)
        for (int j = 0; j < OCV_HARRIS_BLOCK; j++) {
            const int y = y0 - r + i, x = x0 - r + j;
            const int Ix = (im.at(y, x + 1) - im.at(y, x - 1)) * 2 + (im.at(y - 1, x + 1) - im.at(y - 1, x - 1)) +
                           (im.at(y + 1, x + 1) - im.at(y + 1, x - 1));
            const int Iy = (im.at(y + 1, x) - im.at(y - 1, x)) * 2 + (im.at(y + 1, x - 1) - im.at(y - 1, x - 1)) +
                           (im.at(y + 1, x + 1) - im.at(y - 1, x + 1));
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    return ((float)a * b - (float)c * c - OCV_HARRIS_K * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
}

// cv::ORB::detect on one image (a grid cell's sub-image): pyramid (level 0 =
// the image, level l = resize of level l-1 to cvRound(size / scale_l)), per
// level FAST(fastThreshold, nonmax) -> runByImageBorder(edgeThreshold) ->
// retainBest(2 * quota) with octave / size set; Harris responses; per level
// retainBest(quota) on them; ICAngles (unblurred level, umax of half patch
// 15); pt *= scale. Keypoint order: level-major, retainBest's permutation.
void orbcv_detect(const uint8_t* base, int stride, int rows, int cols, int threshold, std::vector<KP>& out,
                  const std::vector<int>& umax) {
    out.clear();
    if (rows <= 0 || cols <= 0) return;
    const std::vector<int> quota = orbcv_quotas(OCV_NFEATURES, OCV_NLEVELS);
    std::vector<Img> pyr(OCV_NLEVELS);
    pyr[0].w = cols;
    pyr[0].h = rows;
    pyr[0].px.resize((size_t)rows * cols);
    for (int y = 0; y < rows; y++) memcpy(&pyr[0].px[(size_t)y * cols], base + (size_t)y * stride, cols);
    for (int l = 1; l < OCV_NLEVELS; l++) {
        const float inv = 1.0f / orbcv_scale(l);
        resize_linear(pyr[l - 1], pyr[l], cvRound((float)cols * inv), cvRound((float)rows * inv));
    }
    std::vector<std::vector<KP>> lv(OCV_NLEVELS);
    for (int l = 0; l < OCV_NLEVELS; l++) {
        const Img& im = pyr[l];
        fast_roi(im.px.data(), im.w, im.h, im.w, threshold, lv[l]);
        run_by_image_border(lv[l], im.w, im.h, OCV_EDGE);
        retain_best(lv[l], 2 * quota[l]);
        const float sf = orbcv_scale(l);
        for (KP& k : lv[l]) {
            k.octave = l;
            k.size = OCV_PATCH * sf;
        }
    }
    for (int l = 0; l < OCV_NLEVELS; l++) {
        for (KP& k : lv[l]) k.response = harris_response(pyr[l], cvRound(k.x), cvRound(k.y));
        retain_best(lv[l], quota[l]);
        for (KP& k : lv[l]) k.angle = ic_angle(pyr[l], k.x, k.y, umax);
        const float sf = orbcv_scale(l);
        for (KP& k : lv[l]) {
            k.x *= sf;
            k.y *= sf;
        }
        out.insert(out.end(), lv[l].begin(), lv[l].end());
    }
}

int adaptive_orb_cell_detect(const uint8_t* base, int stride, int rows, int cols, const odo_adaptive_params& p,
                             double& thresh, std::vector<KP>& kps, const std::vector<int>& umax) {
    int iterCount = p.escape_iters;
    int t_used = 0;
    do {  // VideoDynamicAdaptedFeatureDetector::detect (videodynamicadaptedfeaturedetector.cpp:24-44)
        kps.clear();
        t_used = (int)thresh;  // static_cast<int>(mThresh) (detectoradjuster.cpp:29)
        orbcv_detect(base, stride, rows, cols, t_used, kps, umax);
        const int found = (int)kps.size();
        if (found < p.cell_min) {
            thresh *= p.decrease_factor;
            if (thresh < p.min_thresh) thresh = p.min_thresh;
        } else if (found > p.cell_max) {
            thresh *= p.increase_factor;
            if (thresh > p.max_thresh) thresh = p.max_thresh;
            break;
        } else
            break;
        iterCount--;
    } while (iterCount > 0 && (thresh > p.min_thresh) && (thresh < p.max_thresh));
    return std::min(std::max(t_used, 0), 255);
}

void adaptive_orb_grid_detect(const uint8_t* gray, int w, int h, const odo_adaptive_params& p, double* thresh,
                              std::vector<KP>& out, int* t_used) {
    const int R = p.grid_rows, C = p.grid_cols, E = p.edge_threshold;
    const int maxPerCell = p.max_total_keypoints / (R * C);
    const std::vector<int> umax = make_tables(odo_orb_params{1000, 1.2f, 8, 20, 7}).umax;  // same 15-radius table
    std::vector<std::vector<KP>> sub(R * C);
    for (int i = 0; i < R; ++i) {
        const int rs = std::max((i * h) / R - E, 0), re = std::min(h, ((i + 1) * h) / R + E);
        for (int j = 0; j < C; ++j) {
            const int cs = std::max((j * w) / C - E, 0), ce = std::min(w, ((j + 1) * w) / C + E);
            const int t = adaptive_orb_cell_detect(gray + (size_t)rs * w + cs, w, re - rs, ce - cs, p,
                                                   thresh[j + i * C], sub[j + i * C], umax);
            if (t_used) t_used[j + i * C] = t;
            keep_strongest(maxPerCell, sub[j + i * C]);
        }
    }
    out.clear();
    for (int i = 0; i < R; ++i) {
        const int rs = std::max((i * h) / R - E, 0);
        for (int j = 0; j < C; ++j) {
            const int cs = std::max((j * w) / C - E, 0);
            for (KP& k : sub[j + i * C]) {
                k.x += cs;
                k.y += rs;
            }
            out.insert(out.end(), sub[j + i * C].begin(), sub[j + i * C].end());
        }
    }
}

// cv::ORB::compute on keypoints with octaves (orb.cpp, !do_keypoints):
// runByImageBorder(31) on the image; keypoints grouped by octave (stable, the
// !sortedByLevel regrouping); pyramid of the whole image with the getScale
// sizes; each level blurred in place inside the bordered pyramid (GaussianBlur
// 7x7 REFLECT_101 on the level ROI), so a pattern sample that falls outside
// the level reads the unblurred REFLECT_101 border; centre =
// cvRound(pt / layerScale) (computeOrbDescriptors).
void orb_compute_provided_levels(const uint8_t* gray, int w, int h, std::vector<KP>& kps,
                                 std::vector<uint8_t>& desc) {
    run_by_image_border(kps, w, h, 31);
    std::stable_sort(kps.begin(), kps.end(), [](const KP& a, const KP& b) { return a.octave < b.octave; });
    desc.assign(kps.size() * 32, 0);
    if (kps.empty()) return;
    int nlev = 0;
    for (const KP& k : kps) nlev = std::max(nlev, k.octave + 1);
    std::vector<Img> pyr(nlev), blr(nlev);
    pyr[0].w = w;
    pyr[0].h = h;
    pyr[0].px.assign(gray, gray + (size_t)w * h);
    for (int l = 1; l < nlev; l++) {
        const float inv = 1.0f / orbcv_scale(l);
        resize_linear(pyr[l - 1], pyr[l], cvRound((float)w * inv), cvRound((float)h * inv));
    }
    for (int l = 0; l < nlev; l++) gaussian_blur(pyr[l], blr[l]);
    for (size_t i = 0; i < kps.size(); i++) {
        const KP& k = kps[i];
        const Img &B = blr[k.octave], &U = pyr[k.octave];
        const float sc = 1.f / orbcv_scale(k.octave);
        const int cy = cvRound(k.y * sc), cx = cvRound(k.x * sc);
        const float ang = k.angle * (float)(M_PI / 180.f);
        const float a = (float)cos((double)ang), b = (float)sin((double)ang);
        const int8_t* pattern = ODO_ORB_PATTERN;
        auto value = [&](int idx) {
            const float px = (float)pattern[2 * idx], py = (float)pattern[2 * idx + 1];
            const int yy = cy + cvRound(px * b + py * a), xx = cx + cvRound(px * a - py * b);
            if (yy >= 0 && yy < B.h && xx >= 0 && xx < B.w) return (int)B.at(yy, xx);
            return (int)U.at(reflect101(yy, U.h), reflect101(xx, U.w));
        };
        for (int j = 0; j < 32; ++j, pattern += 32) {
            int val = 0;
            for (int bit = 0; bit < 8; bit++) val |= (value(2 * bit) < value(2 * bit + 1)) << bit;
            desc[i * 32 + j] = (uint8_t)val;
        }
    }
}

int adaptive_orb_extract(const uint8_t* gray, int w, int h, const odo_adaptive_params& p, double* thresh,
                         std::vector<KP>& kps, std::vector<uint8_t>& desc, int* t_used) {
    adaptive_orb_grid_detect(gray, w, h, p, thresh, kps, t_used);
    if ((int)kps.size() > p.retain_best) retain_best(kps, p.retain_best);  // extractor.cpp:45-46
    orb_compute_provided_levels(gray, w, h, kps, desc);
    return (int)kps.size();
}

}  // namespace

// ================================================================ C API
extern "C" {

void oracle_bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray) {
    bgr2gray(bgr, w, h, stride, gray);
}

void oracle_depth_to_f32(const uint16_t* d, int n, float factor, float* z) {
    // Mat::convertTo(CV_32F, alpha): dst = (float)src * (float)alpha + 0.f
    const float a = (float)(double)factor;
    for (int i = 0; i < n; i++) z[i] = (float)d[i] * a + 0.0f;
}

int oracle_level_sizes(const odo_orb_params* p, int w, int h, int* lw, int* lh, float* scale,
                       int* quota) {
    Tables t = make_tables(*p);
    for (int l = 0; l < p->nlevels; l++) {
        lw[l] = cvRound((float)w * t.inv_scale[l]);
        lh[l] = cvRound((float)h * t.inv_scale[l]);
        if (scale) scale[l] = t.scale[l];
        if (quota) quota[l] = t.quota[l];
    }
    return p->nlevels;
}

int oracle_umax(int* umax16) {
    odo_orb_params p{1000, 1.2f, 8, 20, 7};
    Tables t = make_tables(p);
    for (int i = 0; i < 16; i++) umax16[i] = t.umax[i];
    return 16;
}

int oracle_pyramid(const uint8_t* gray, int w, int h, const odo_orb_params* p, uint8_t* out) {
    Extractor ex(*p);
    ex.compute_pyramid(gray, w, h);
    size_t off = 0;
    for (auto& im : ex.pyr) {
        memcpy(out + off, im.px.data(), im.px.size());
        off += im.px.size();
    }
    return (int)off;
}

int oracle_fast_level(const uint8_t* img, int w, int h, int ini_th, int min_th, orb_kp* out, int cap) {
    Img im;
    im.w = w;
    im.h = h;
    im.px.assign(img, img + (size_t)w * h);
    std::vector<KP> c;
    fast_level(im, ini_th, min_th, c);
    int n = std::min((int)c.size(), cap);
    for (int i = 0; i < n; i++)
        out[i] = orb_kp{c[i].x, c[i].y, c[i].size, c[i].angle, c[i].response, c[i].octave, c[i].class_id};
    return (int)c.size();
}

int oracle_octree(const orb_kp* keys, int n, int minX, int maxX, int minY, int maxY, int N,
                  orb_kp* out, int cap) {
    std::vector<KP> k(n);
    for (int i = 0; i < n; i++)
        k[i] = KP{keys[i].x, keys[i].y, keys[i].size, keys[i].angle, keys[i].response, keys[i].octave,
                  keys[i].class_id};
    if (n == 0) return 0;
    std::vector<KP> r = distribute_octree(k, minX, maxX, minY, maxY, N);
    int m = std::min((int)r.size(), cap);
    for (int i = 0; i < m; i++)
        out[i] = orb_kp{r[i].x, r[i].y, r[i].size, r[i].angle, r[i].response, r[i].octave, r[i].class_id};
    return (int)r.size();
}

void oracle_blur(const uint8_t* img, int w, int h, uint8_t* out) {
    Img a, b;
    a.w = w;
    a.h = h;
    a.px.assign(img, img + (size_t)w * h);
    gaussian_blur(a, b);
    memcpy(out, b.px.data(), b.px.size());
}

float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }

int oracle_orb_extract(const uint8_t* gray, int w, int h, const odo_orb_params* p, orb_kp* kps,
                       uint8_t* desc, int cap) {
    Extractor ex(*p);
    ex.ini_th = p->ini_th_fast;
    ex.min_th = p->min_th_fast;
    std::vector<KP> out;
    std::vector<uint8_t> d;
    int n = ex.run(gray, w, h, out, d);
    int m = std::min(n, cap);
    for (int i = 0; i < m; i++)
        kps[i] = orb_kp{out[i].x, out[i].y, out[i].size, out[i].angle, out[i].response, out[i].octave,
                        out[i].class_id};
    if (desc) memcpy(desc, d.data(), (size_t)m * 32);
    return n;
}

static void kp_out(const std::vector<KP>& v, orb_kp* out, int cap) {
    const int m = std::min((int)v.size(), cap);
    for (int i = 0; i < m; i++)
        out[i] = orb_kp{v[i].x, v[i].y, v[i].size, v[i].angle, v[i].response, v[i].octave, v[i].class_id};
}

void oracle_adaptive_default(odo_adaptive_params* p) {
    // Extractor::CreateAdaptiveDetector (extractor.cpp:55-77) + nFeatures (common.h:77)
    const int minFeatures = 600;
    const int maxFeatures = minFeatures * 1.7;
    const int cells = 3 * 3;
    *p = odo_adaptive_params{3, 3, 31, maxFeatures, (int)round(minFeatures / (float)cells),
                             (int)round(maxFeatures / (float)cells), 5, 20, 2, 10000, 1.3, 0.7, 1000};
}

int oracle_adaptive_detect(const uint8_t* gray, int w, int h, const odo_adaptive_params* p, double* thresh,
                           orb_kp* out, int cap, int* t_used) {
    std::vector<KP> k;
    adaptive_grid_detect(gray, w, h, *p, thresh, k, t_used);
    kp_out(k, out, cap);
    return (int)k.size();
}

int oracle_fast_roi(const uint8_t* gray, int stride, int rows, int cols, int threshold, orb_kp* out, int cap) {
    std::vector<KP> k;
    fast_roi(gray, stride, rows, cols, threshold, k);
    kp_out(k, out, cap);
    return (int)k.size();
}

int oracle_adaptive_extract(const uint8_t* gray, int w, int h, const odo_adaptive_params* p, double* thresh,
                            orb_kp* kps, uint8_t* desc, int cap, int* t_used) {
    std::vector<KP> k;
    std::vector<uint8_t> d;
    const int n = adaptive_extract(gray, w, h, *p, thresh, k, d, t_used);
    kp_out(k, kps, cap);
    if (desc) memcpy(desc, d.data(), (size_t)std::min(n, cap) * 32);
    return n;
}

int oracle_adaptive_orb_extract(const uint8_t* gray, int w, int h, const odo_adaptive_params* p, double* thresh,
                                orb_kp* kps, uint8_t* desc, int cap, int* t_used) {
    std::vector<KP> k;
    std::vector<uint8_t> d;
    const int n = adaptive_orb_extract(gray, w, h, *p, thresh, k, d, t_used);
    kp_out(k, kps, cap);
    if (desc) memcpy(desc, d.data(), (size_t)std::min(n, cap) * 32);
    return n;
}

int oracle_adaptive_orb_detect(const uint8_t* gray, int w, int h, const odo_adaptive_params* p, double* thresh,
                               orb_kp* out, int cap, int* t_used) {
    std::vector<KP> k;
    adaptive_orb_grid_detect(gray, w, h, *p, thresh, k, t_used);
    kp_out(k, out, cap);
    return (int)k.size();
}

int oracle_orbcv_detect(const uint8_t* img, int stride, int rows, int cols, int threshold, orb_kp* out, int cap) {
    std::vector<KP> k;
    const std::vector<int> umax = make_tables(odo_orb_params{1000, 1.2f, 8, 20, 7}).umax;
    orbcv_detect(img, stride, rows, cols, threshold, k, umax);
    kp_out(k, out, cap);
    return (int)k.size();
}

float oracle_harris(const uint8_t* img, int w, int h, int x, int y) {
    Img im;
    im.w = w;
    im.h = h;
    im.px.assign(img, img + (size_t)w * h);
    return harris_response(im, x, y);
}

int oracle_orbcv_levels(int w, int h, int* lw, int* lh, float* scale, int* quota) {
    const std::vector<int> q = orbcv_quotas(OCV_NFEATURES, OCV_NLEVELS);
    for (int l = 0; l < OCV_NLEVELS; l++) {
        const float inv = 1.0f / orbcv_scale(l);
        lw[l] = cvRound((float)w * inv);
        lh[l] = cvRound((float)h * inv);
        scale[l] = orbcv_scale(l);
        quota[l] = q[l];
    }
    return OCV_NLEVELS;
}

// std::nth_element / partition helpers on packed (score<<24 | y<<12 | x)
// keys, compared by score only (the GPU selection's test hooks)
void oracle_nth_element_score(uint32_t* a, int n, int nth) {
    std::nth_element(a, a + nth, a + n, [](uint32_t x, uint32_t y) { return (x >> 24) > (y >> 24); });
}

int oracle_retain_best_score(uint32_t* a, int n, int n_points) {
    std::vector<KP> k(n);
    for (int i = 0; i < n; i++) k[i] = KP{(float)(a[i] & 0xfff), (float)((a[i] >> 12) & 0xfff), 7.f, -1.f,
                                          (float)(a[i] >> 24), 0, -1};
    retain_best(k, n_points);
    for (size_t i = 0; i < k.size(); i++)
        a[i] = ((uint32_t)k[i].response << 24) | ((uint32_t)k[i].y << 12) | (uint32_t)k[i].x;
    return (int)k.size();
}

}  // extern "C"
