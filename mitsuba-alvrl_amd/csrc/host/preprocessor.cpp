// preprocessor.cpp -- LightSlice slicing and representative sampling on the
// host (Preprocessor.cpp:66-121, 779-827, 1130-1525).  The priority queue is a
// std::vector driven by std::push_heap / std::pop_heap, which is what
// boost::heap::priority_queue is built on; its iteration order (the vector
// order) decides the slice numbering exactly as in the reference.
#include "preprocessor.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace alvrl {
namespace host {

namespace {
constexpr uint32_t kDomReps = 4u;

void philox(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

struct Stream {
    uint32_t seed, pass, dom, a, b, c, k = 0, blk = 0xFFFFFFFFu;
    uint32_t buf[4];
    float next()
    {
        const uint32_t bl = k >> 2;
        if (bl != blk) {
            const uint32_t ctr[4] = {a, b, bl, (dom << 24) | (c & 0xFFFFFFu)};
            const uint32_t key[2] = {seed, pass};
            philox(ctr, key, buf);
            blk = bl;
        }
        union { uint32_t u; float f; } x;
        x.u = (buf[k & 3] >> 9) | 0x3f800000u;
        ++k;
        return x.f - 1.0f;
    }
};

float slice_distance(V3 p1, V3 d1, V3 p2, V3 d2)   // Preprocessor.cpp:1230-1234
{
    const float dx = p1.x - p2.x, dy = p1.y - p2.y, dz = p1.z - p2.z;
    const float ex = d1.x - d2.x, ey = d1.y - d2.y, ez = d1.z - d2.z;
    return std::sqrt((dx * dx + dy * dy + dz * dz) + (ex * ex + ey * ey + ez * ez));
}

void find_split_point(V3 mx, V3 mn, unsigned char* dim, float* split, float* extent)   // :1451-1487
{
    const float dx = mx.x - mn.x, dy = mx.y - mn.y, dz = mx.z - mn.z;
    if (dx == 0 && dy == 0 && dz == 0) {
        *extent = 0; *dim = 0; *split = std::numeric_limits<float>::quiet_NaN();
        return;
    }
    if (dx > dy) {
        if (dx > dz) { *dim = 0; *split = (float)(mn.x + 0.5 * dx); *extent = dx; }
        else { *dim = 2; *split = (float)(mn.z + 0.5 * dz); *extent = dz; }
    } else {
        if (dy > dz) { *dim = 1; *split = (float)(mn.y + 0.5 * dy); *extent = dy; }
        else { *dim = 2; *split = (float)(mn.z + 0.5 * dz); *extent = dz; }
    }
}

struct SliceNode {   // :1295-1341
    uint32_t minInd, maxInd;
    float distance;
    unsigned char dim;
    float split;
    V3 posC, dirC;
    bool operator<(const SliceNode& o) const { return distance < o.distance; }
};

bool make_node(SliceNode* sn, uint32_t minI, uint32_t maxI, const std::vector<V3>& pos,
               const std::vector<V3>& dir, const std::vector<uint32_t>& idx)
{
    sn->minInd = minI; sn->maxInd = maxI;
    if (minI >= maxI) return false;
    const float nan = std::numeric_limits<float>::quiet_NaN();
    if (minI + 1 == maxI) {
        sn->distance = 0; sn->dim = 0; sn->split = nan;
        sn->posC = v3(nan, nan, nan); sn->dirC = sn->posC;
        return true;
    }
    const float inf = std::numeric_limits<float>::infinity();
    V3 mxp = v3(-inf, -inf, -inf), mnp = v3(inf, inf, inf), mxd = mxp, mnd = mnp;
    for (uint32_t i = minI; i < maxI; i++) {
        const V3 p = pos[idx[i]], d = dir[idx[i]];
        if (p.x < mnp.x) mnp.x = p.x;
        if (p.y < mnp.y) mnp.y = p.y;
        if (p.z < mnp.z) mnp.z = p.z;
        if (p.x > mxp.x) mxp.x = p.x;
        if (p.y > mxp.y) mxp.y = p.y;
        if (p.z > mxp.z) mxp.z = p.z;
        if (d.x < mnd.x) mnd.x = d.x;
        if (d.y < mnd.y) mnd.y = d.y;
        if (d.z < mnd.z) mnd.z = d.z;
        if (d.x > mxd.x) mxd.x = d.x;
        if (d.y > mxd.y) mxd.y = d.y;
        if (d.z > mxd.z) mxd.z = d.z;
    }
    sn->distance = slice_distance(mnp, mnd, mxp, mxd);
    unsigned char dp, dd;
    float sp, sd, ep, ed;
    find_split_point(mxp, mnp, &dp, &sp, &ep);
    find_split_point(mxd, mnd, &dd, &sd, &ed);
    if (ep == 0 && ed == 0) return false;   // "findSplit: min equal to max!"
    if (ep > ed) { sn->dim = dp; sn->split = sp; }
    else { sn->dim = (unsigned char)(3 + dd); sn->split = sd; }
    sn->posC = v3(mnp.x + 0.5f * (mxp.x - mnp.x), mnp.y + 0.5f * (mxp.y - mnp.y), mnp.z + 0.5f * (mxp.z - mnp.z));
    sn->dirC = v3(mnd.x + 0.5f * (mxd.x - mnd.x), mnd.y + 0.5f * (mxd.y - mnd.y), mnd.z + 0.5f * (mxd.z - mnd.z));
    return true;
}

inline bool is_larger(V3 p, V3 d, int dim, float split)   // :1420-1430
{
    switch (dim) {
    case 0: return p.x > split;
    case 1: return p.y > split;
    case 2: return p.z > split;
    case 3: return d.x > split;
    case 4: return d.y > split;
    default: return d.z > split;
    }
}

inline bool finite3(V3 p) { return std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z); }

}  // namespace

std::vector<uint32_t> Preprocessor::build_slices(const SmokeBox& s, const float* recs)
{
    const int W = s.width, H = s.height;
    m_W = W; m_H = H;
    const uint32_t n = (uint32_t)W * (uint32_t)H;
    std::vector<V3> pos(n), dir(n);
    const float directionScale = s.scene_diagonal() / 8 * m_p.slice_curvature_factor;   // :1137
    const float nan = std::numeric_limits<float>::quiet_NaN();
    for (int i = 0; i < W; i++) {          // pixel order: x outer, y inner (:1140-1141)
        for (int j = 0; j < H; j++) {
            float own[kRecWords];
            const float* rec = own;
            if (recs) rec = recs + kRecWords * ((size_t)j * W + i);
            else s.make_slice_record(i, j, own);
            uint32_t flags;
            std::memcpy(&flags, &rec[15], 4);
            const uint32_t k = (uint32_t)i * H + j;
            if (flags & 1u) {
                pos[k] = v3(rec[6], rec[7], rec[8]);
                dir[k] = v3(directionScale * rec[9], directionScale * rec[10], directionScale * rec[11]);
            } else {
                pos[k] = v3(nan, nan, nan);
                dir[k] = pos[k];
            }
        }
    }
    std::vector<uint32_t> idx(n), p2s(n, 0xFFFFFFFFu);
    for (uint32_t i = 0; i < n; i++) idx[i] = i;
    uint32_t first = 0;   // getSlices: infinite gather points to the front (:1206-1221)
    while (first < n && !finite3(pos[first])) first++;
    for (uint32_t i = first + 1; i < n; i++)
        if (!finite3(pos[i])) { idx[i] = idx[first]; idx[first] = i; first++; }
    std::vector<SliceNode> pq;
    bool ok = true;
    if (first < n) {
        SliceNode sn;
        ok &= make_node(&sn, first, n, pos, dir, idx);
        pq.push_back(sn);
        std::push_heap(pq.begin(), pq.end());
        while (ok && pq.size() < m_p.target_num_slices && pq.front().distance > 0) {
            std::pop_heap(pq.begin(), pq.end());
            const SliceNode top = pq.back();
            pq.pop_back();
            const size_t lo = top.minInd, hi = top.maxInd - 1;
            size_t i = lo - 1, j = hi + 1;
            while (true) {   // :1373-1393
                while (true) { i++; if (is_larger(pos[idx[i]], dir[idx[i]], top.dim, top.split) || i == hi) break; }
                while (true) { j--; if (!is_larger(pos[idx[j]], dir[idx[j]], top.dim, top.split) || j == lo) break; }
                if (i >= j) break;
                std::swap(idx[i], idx[j]);
            }
            SliceNode a, b;
            ok &= make_node(&a, top.minInd, (uint32_t)(j + 1), pos, dir, idx);
            ok &= make_node(&b, (uint32_t)(j + 1), top.maxInd, pos, dir, idx);
            pq.push_back(a); std::push_heap(pq.begin(), pq.end());
            pq.push_back(b); std::push_heap(pq.begin(), pq.end());
        }
    }
    if (!ok) throw std::runtime_error("buildSlices: degenerate slice split");
    m_lo.clear(); m_hi.clear(); m_posC.clear(); m_dirC.clear();
    for (size_t k = 0; k < pq.size(); k++) {   // save the slices in heap-vector order (:1400-1417)
        m_lo.push_back(pq[k].minInd); m_hi.push_back(pq[k].maxInd);
        m_posC.push_back(pq[k].posC); m_dirC.push_back(pq[k].dirC);
        for (uint32_t i = pq[k].minInd; i < pq[k].maxInd; i++) p2s[idx[i]] = (uint32_t)k;
    }
    m_idx.swap(idx);
    return p2s;
}

void Preprocessor::sample_slice_mapping(float targetUnder)
{
    const uint32_t ns = num_slices();
    m_rep_off.assign(ns + 1, 0);
    m_rep_pix.clear();
    m_slice_under.assign(ns, 0.0f);
    size_t totalPix = 0, totalRep = 0;
    for (uint32_t s = 0; s < ns; s++) {   // Slice::sampleRepresentativePixels (:66-121)
        m_rep_off[s] = (uint32_t)m_rep_pix.size();
        const size_t np = m_hi[s] - m_lo[s];
        const uint32_t* gp = m_idx.data() + m_lo[s];
        size_t target = (size_t)(0.5 + (double)((float)np / targetUnder));
        if (target < 2) target = std::min((size_t)2, np);
        Stream smp{m_p.seed, m_p.pass, kDomReps, s, 0u, 0u};
        if (np <= target) {
            for (size_t i = 0; i < np; i++) m_rep_pix.push_back(gp[i]);
        } else if (np <= 2 * target) {
            std::vector<uint32_t> ind(np);
            for (size_t i = 0; i < np; i++) ind[i] = (uint32_t)i;
            for (size_t i = np - 1; i > 0; i--) {
                const size_t k = (size_t)((float)(i + 1) * smp.next());
                std::swap(ind[i], ind[k]);
            }
            for (size_t i = 0; i < target; i++) m_rep_pix.push_back(gp[ind[i]]);
        } else {
            std::vector<uint32_t> ind(target);
            size_t n = 0;
            while (n < target) {
                bool unique;
                do {
                    ind[n] = (uint32_t)(smp.next() * (float)np);
                    unique = true;
                    for (size_t i = 0; i < n; i++) if (ind[i] == ind[n]) { unique = false; break; }
                } while (!unique);
                n++;
            }
            for (size_t i = 0; i < target; i++) m_rep_pix.push_back(gp[ind[i]]);
        }
        const size_t nrep = m_rep_pix.size() - m_rep_off[s];
        m_slice_under[s] = (float)nrep / (float)np;
        totalRep += nrep; totalPix += np;
    }
    m_rep_off[ns] = (uint32_t)m_rep_pix.size();
    // buildLocalities (:1241-1293)
    m_loc.assign(ns, {});
    const uint32_t nc = m_p.neighbour_count;
    if (ns <= nc) {
        for (uint32_t i = 0; i < ns; i++)
            for (uint32_t j = 0; j < ns; j++)
                if (i != j) m_loc[i].insert({j, slice_distance(m_posC[i], m_dirC[i], m_posC[j], m_dirC[j])});
    } else if (nc > 0) {
        std::vector<float> dist(nc);
        std::vector<uint32_t> ind(nc, 0);
        uint32_t maxInd = 0;   // not reset per slice, as in the reference (:1263)
        for (uint32_t i = 0; i < ns; i++) {
            std::fill(dist.begin(), dist.end(), std::numeric_limits<float>::infinity());
            for (uint32_t j = 0; j < ns; j++) {
                if (i == j) continue;
                const float d = slice_distance(m_posC[i], m_dirC[i], m_posC[j], m_dirC[j]);
                if (d < dist[maxInd]) {
                    dist[maxInd] = d; ind[maxInd] = j;
                    for (uint32_t k = 0; k < nc; k++) if (dist[k] > dist[maxInd]) maxInd = k;
                }
            }
            for (uint32_t x = 0; x < nc; x++) m_loc[i].insert({ind[x], dist[x]});
        }
    }
    m_global_under = (float)totalRep / (float)totalPix;
}

void Preprocessor::local_matrix(uint32_t i, std::vector<uint32_t>* rows, std::vector<double>* w) const
{
    rows->clear(); w->clear();
    const uint32_t r0 = m_rep_off[i], r1 = m_rep_off[i + 1], ni = r1 - r0;
    for (uint32_t r = r0; r < r1; r++) rows->push_back(r);
    if (m_p.neighbour_weight <= 0) {
        for (uint32_t k = 0; k < ni; k++) w->push_back(1.0 / (double)ni);
        return;
    }
    std::vector<float> nw;
    float summed = 0;
    for (const auto& loc : m_loc[i]) {
        for (uint32_t r = m_rep_off[loc.first]; r < m_rep_off[loc.first + 1]; r++) rows->push_back(r);
        nw.push_back((float)(1.0 / (double)loc.second));
        summed += nw.back();
    }
    const float nwgt = m_p.neighbour_weight;
    const float sliceWeight = summed * (1 - nwgt) / nwgt;
    const float normalization = 1 / (sliceWeight + summed);
    for (uint32_t k = 0; k < ni; k++) w->push_back((double)(sliceWeight * normalization / (float)ni));
    size_t q = 0;
    for (const auto& loc : m_loc[i]) {
        const uint32_t cnt = m_rep_off[loc.first + 1] - m_rep_off[loc.first];
        for (uint32_t k = 0; k < cnt; k++) w->push_back((double)(nw[q] * normalization / (float)cnt));
        q++;
    }
}

}  // namespace host
}  // namespace alvrl
