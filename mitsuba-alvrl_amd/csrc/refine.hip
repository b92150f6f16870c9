// refine.hip -- LightSlice cluster refinement on gfx950.
//
// Restates class Preprocessor::Clustering (src/integrators/vrl/Preprocessor.cpp:
// 287-720) and its helpers (calculateColumnWeigths :985-1008,
// calculateUnclusteredVariance :1022-1048, calculateClusterVariance
// :1058-1120, weightedSample :1534-1580) as ONE persistent workgroup per
// clustering job (a slice's local matrix L_i, or the fall-back matrix).
//
// Work decomposition inside a job (8 waves):
//  * the best-first control flow (priority queue, singleton list, snapshot /
//    restore, convergence constants) runs on lane 0 of wave 0, exactly in the
//    reference's order; the heap is std::push_heap/pop_heap's algorithm;
//  * column work (column weights, projections) runs one wave per VRL column,
//    lanes over the local-matrix rows, with the deterministic wave order that
//    oracle/alvrl_preproc.c uses (lane l sums rows l, l+64, ...; halving tree);
//  * the forward / reverse cluster-variance recurrences (:1075-1109) are
//    sequential along the cluster and parallel over rows (one lane per row),
//    processed in chunks of 64 prefixes; the per-prefix inner products over
//    rows are again one wave each;
//  * the projection sort is a bitonic sort in LDS (<= 4096 keys) or a 1-bit
//    LSD split radix sort in global scratch; keys are (orderable float, vrl),
//    unique, so any correct sort reproduces std::sort on std::pair.
// This file is compiled with -ffp-contract=off: every double/float operation
// is the same IEEE operation the oracle performs, so the resulting cluster
// indices and weights are bit-identical to the CPU restatement.
#include "vrl_device.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

namespace alvrl {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kCH = 8;                                      // columns per variance chunk (per direction)
constexpr int kGT = kThreads / 2;                           // threads per variance direction
constexpr uint32_t kPoolBytes = 152 * 1024;                 // dynamic LDS: sort keys / variance chunks
constexpr int kBitonicMax = 16384;                          // 8-byte keys sorted in the pool
constexpr uint32_t kDomCluster = 5u;

struct CNode { float uvar, ivar; uint32_t begin, end; };

// Speculative splits (team mode).  A split's result is a function of its
// cluster alone (its draws are keyed by the cluster range, the sort is a
// total order), and the live clusters are disjoint ranges of vrls.  Helper
// workgroups therefore split clusters near the top of the heap ahead of the
// leader into range-indexed side buffers; the leader, which runs the
// reference's control flow unchanged, commits a finished result when it pops
// that cluster (or claims a queued one, or splits an unqueued one itself).
// v_first / v_last: the ids at the first and last sorted positions, so that a
// commit pushes a single child without reading its id back from team.spec
struct SplitRes { uint32_t idx; int err; float fsu, fsi, feu, fei; uint32_t v_first, v_last; };
struct SplitWs {                      // a workgroup's private split scratch
    float* dir;
    double* st;
    double* bufM;
    unsigned long long* keys0;
    unsigned long long* keys1;
    float* fsu; float* fsi; float* feu; float* fei;
    double* carry;                    // [2][N][2] row-group sums of the v3 engine (null: rows <= 256)
};
struct Team {
    uint32_t helpers;                 // workgroups besides the leader (0 = off)
    uint32_t* spec;                   // [N] sorted ranges of speculative splits, by position
    unsigned long long* state;        // [N] by cluster begin: (end << 3) | kSt*
    SplitRes* res;                    // [N] by cluster begin
    unsigned long long* queue;        // [kQueue] (begin << 32) | end
    uint32_t* ctl;                    // head, tail, stop
    const SplitWs* ws;                // [helpers]
};
enum : uint32_t { kStNone = 0, kStQueued = 1, kStRunning = 2, kStDone = 3, kStLeader = 4 };
// Split parts.  A large split's two variance passes over a group of row
// blocks are independent of every other (pass, group): each writes the 64-row
// block totals of its per-column prefix terms, and the owner of the split
// adds them in ascending block order afterwards (wsum_blk's order, so the
// prefixes are those of the one-workgroup engine bit for bit).  The owner
// publishes the parts on a slot of the part board; idle workgroups (helpers,
// roamers, a leader waiting for a helper) claim them.  Nothing a claimer does
// waits for anyone, so the owner's wait for its claimed parts ends.
struct PartJob {
    const unsigned long long* roff;   // the job's row layout (JobDev's)
    const uint32_t* rstride;
    unsigned long long off0;
    uint32_t stride0;
    int contig;
    const double* locw;
    uint32_t nrows;
    uint32_t kind;                    // kPartVar: variance passes; kPartProj: projections
    const unsigned long long* cw;     // kPartVar: the cluster's (weight << 32 | vrl), column order (the owner's keys1)
    const uint32_t* ids;              // kPartProj: the cluster's columns, their split direction, the keys out
    const float* dir;
    unsigned long long* keys;
    uint32_t m;                       // columns
    uint32_t nblk, pblk, np;          // 64-row blocks, blocks per part (kPartVar), parts
    uint32_t cpp;                     // kPartProj / kPartColw: columns per part
    float* colw;                      // kPartColw: the column weights out
    uint32_t c0;                      // kPartColw: the first column (parts cover [c0, m))
    double* st;                       // kPartInit: the rows' final (sum, M, V) states out (the owner's J.st)
    double* wsum;                     // kPartInit: the total column weight (the slot's)
};
enum : uint32_t { kPartVar = 0, kPartProj = 1, kPartColw = 2, kPartInit = 3 };
struct PartSlot {
    unsigned long long word;          // generation << 32 | parts << 16 | parts claimed
    uint32_t busy;                    // an owner holds the slot
    uint32_t done;                    // parts finished (each after a release)
    uint32_t err;                     // a part's engine error
    uint32_t pad;
    double wsum;                      // kPartInit: the pass's total column weight
    double* T;                        // [pass][u|i][block][column] block totals (fixed per slot)
    PartJob pj;
};
// A cluster born from a committed speculative split has its vrls in team.spec
// already (the parent's output, which the leader copied to vrls): bit 63 of
// its state word and bit 31 of its queue entry's end say so, and its helper
// splits team.spec in place instead of copying vrls, which the leader then
// need not release.
constexpr unsigned long long kStSpecBit = 1ull << 63;
constexpr uint32_t kQSpecBit = 1u << 31;
constexpr uint32_t kQueue = 1024;
constexpr int kSpecWidthMax = 256;      // heap entries a leader examines per enqueue (ALVRL_SPEC_WIDTH)
// The leader's heap nodes carry two flags in the top bits of `end`: queued by
// this leader (a helper may be on it: its state word decides), and its vrls
// already in team.spec (a committed speculative split's child).  Queueing
// needs no state-word loads; every other reader strips them (kEndMask).
constexpr uint32_t kEndQ = 1u << 31;
constexpr uint32_t kEndS = 1u << 30;
constexpr uint32_t kEndMask = kEndS - 1u;

struct JobDev {
    // entry (vrl v, local row r) of R is Rt[roff[r] + v * rstride[r]] (float2
    // units); contig: roff[r] == off0 + r and rstride[r] == stride0 for all r
    const unsigned long long* roff;
    const uint32_t* rstride;
    unsigned long long off0;
    uint32_t stride0;
    int contig;
    const double* locw;
    uint32_t nrows;
    float pixel_under, undersampling, depth_correction;
    int do_refine;
    uint32_t stage_refine, stage_sample;
    // workspace (device, sized by the host)
    uint32_t* vrls;
    float* colw;
    CNode* heap;
    CNode* sh_heap;
    uint32_t* singles;
    uint32_t* sh_singles;
    float* dir;
    unsigned long long* keys0;
    unsigned long long* keys1;
    float* fsu; float* fsi; float* feu; float* fei;
    double* carry;     // [2][N][2]: the v3 engine's block-ordered row sums between row groups (null: rows <= 256)
    double* st;        // 2 x 3 * nrows: sum, M, sumVars per variance direction
    double* bufM;      // 2 x kCH * (nrows | 1): per-row terms when they do not fit in LDS
    double* bufV;
    // outputs
    uint32_t* out_reps;
    float* out_w;
    uint32_t* out_n;
    int* out_refined;
    int* out_err;
    // getVrlsPerCluster (optional): member ids, cluster offsets, cluster count
    uint32_t* out_members;
    uint32_t* out_moff;
    uint32_t* out_nclusters;
    Team team;
};

struct Common {
    const float2* Rt;
    uint64_t ld;
    uint32_t nvrl;
    const uint32_t* init_vrls;
    const uint32_t* init_off;
    uint32_t ninit;
    uint32_t seed, pass;
    unsigned long long* prof;   // per-phase cycle totals (ALVRL_REFINE_PROFILE=1), or null
    unsigned long long* entries;   // [0]: R entries read once per setup pass and split (roofline bytes / 8),
                                   // [1]: of those, the splits' (each split reads them three times)
    uint32_t njobs;                // leaders = blocks [0, njobs); helpers follow, team by team
    uint32_t team;                 // workgroups per job (1 = no speculation)
    uint32_t spec_min;             // smallest cluster worth a speculative split
    uint32_t side_k;               // a waiting leader takes a side task of <= awaited columns * side_k / 16
    int enq_start;                 // also queue candidates right after the pop (before the split)
    unsigned long long spin_ticks; // bound of an idle helper's wait for a task (100 MHz ticks)
    unsigned long long wait_ticks; // bound of a leader's wait for a running helper (100 MHz ticks)
    uint32_t sort_radix_min;       // clusters of at least this many columns: radix8_sort
    uint32_t ws_wg_min;            // clusters of at least this many columns: weighted_sample_wg
    int part_red;                  // variance parts of <= 3 row blocks: trees on reducer waves (ALVRL_PART_RED)
    int colw_all;                  // the leader divides all of a <= 256-row job's column weights (no
                                   // helper half): launches that are not busy (ALVRL_COLW_ALL)
    unsigned long long* tstat;     // team counters (ALVRL_REFINE_TEAM_STATS=1), or null
    unsigned long long* jtime;     // with tstat: per job, wall ticks at start / end of refine / end
    unsigned long long* trace;     // host-mapped per-block (phase << 32 | value), ALVRL_REFINE_TRACE=1
    uint32_t spec_width;           // heap entries examined per enqueue (0 = 2 * helpers + 2)
    uint32_t nroam;                // roaming helpers (after the teams): serve every job's queue
    int var_v3;                    // split variances on variance_split_v3 (ALVRL_VAR_V3=0: the older engine)
    int var_small;                 // splits of <= kSmallMax columns on variance_split_small (ALVRL_VAR_SMALL=0: off)
    int split_fused;               // small splits on split_fused: 2 (default) float2 and means-only staging,
                                   // 1 float2 staging only, 0 off (ALVRL_SPLIT_FUSED)
    int roam_on;                   // finished leaders and helpers roam too (scratch sized for Rmax)
    const SplitWs* roam_ws;        // [nroam] their scratch, sized for the largest job
    const uint32_t* roam_order;    // null: roam from the last job served; else scan jobs in this order
    int early_spec;                // queue the first initial cluster for a helper's split before the
                                   // leader computes the initial clusters' variances (ALVRL_EARLY_SPEC=0: off)
    int team_setup;                // a job's first helper takes half the column weights and the
                                   // unclustered variance off the leader (ALVRL_TEAM_SETUP=0: off)
    int heap_lds;                  // the leader's heap in LDS between its splits (ALVRL_HEAP_LDS=0: off)
    uint32_t* poptr;               // ALVRL_POP_TRACE=1: wall ticks at 7 points of each leader pop of one job
    uint32_t poptr_job, poptr_cap; // the traced job (most rows), records available
    unsigned long long* evlog;     // developer event log (a -DALVRL_EVLOG build, ALVRL_EVLOG=file): 3 words per event
    uint32_t* evlog_n;             // events written
    uint32_t evlog_cap;
    PartSlot* parts;               // the part board (null: splits are never divided)
    uint32_t nslots;               // its slots
    uint32_t part_min;             // smallest split (columns) divided into parts
    uint32_t part_blk;             // 64-row blocks per part (<= 7), jobs of more than 256 rows
    uint32_t part_blk_short;       // ... and of <= 256 rows
    uint32_t part_blk_init;        // ... for an initial cluster's variance (init_parts)
    uint32_t* part_open;           // slots with parts not yet claimed (a hint for idle workgroups)
    uint32_t* idle;                // helpers and roamers waiting for work (parts are published only if some are)
    uint32_t idle_min;             // ... at least this many (0: always)
    uint32_t idle_min_short;       // ... for jobs of <= 256 rows
    uint32_t part_min_tall;        // the same for jobs of more than 256 rows
    uint32_t nbig;                 // slots [0, nbig) hold splits of any size, the rest up to small_cap columns
    uint32_t small_cap;
    uint32_t proj_min;             // smallest split whose projections are divided (0: never)
    uint32_t proj_cpp;             // columns per projection part
    // the jobs as seen with another workgroup's split scratch: views[w * njobs + j] is job j with
    // vrls = team.spec and the scratch of workgroup w (roamers, then helpers, then leaders; k_views)
    const __attribute__((address_space(4))) JobDev* views;
};
// The jobs, their views and Common live in device memory the kernel never
// writes, reached through the constant address space: uniform field reads are
// scalar loads (s_load, the scalar cache), not per-lane vector loads of a
// private copy, whose waits (vmcnt) also waited out every store in flight.
// A function's reference parameters arrive in VGPRs; uni() moves the address
// to SGPRs so that the compiler knows it is uniform.
#define ALVRL_AS4 __attribute__((address_space(4)))
// the leader's pop and quick commit: out of line by default (ALVRL_POP_INLINE=1
// inlines them into k_refine, which drops the wait for every memory operation
// in flight that a call's entry carries)
// developer A/B: the split phases' helpers inlined into split() (no call-entry waits)
#ifdef ALVRL_INL_PROJ
#define ALVRL_PROJ_INL __forceinline__
#else
#define ALVRL_PROJ_INL __noinline__
#endif
// the weighted picks are inlined (C4 refinement -2 ms, profiles/r04/inl/); ALVRL_WS_OUTLINE: a call
#ifdef ALVRL_WS_OUTLINE
#define ALVRL_WS_INL __noinline__
#else
#define ALVRL_WS_INL __forceinline__
#endif
// Small splits and their call frames (profiles/r05/inl/): split() is an inline
// dispatcher that calls split_fused (2-17 callee-saved VGPR stores) or
// split_big (41) directly, so a small split no longer enters the large path's
// frame: C4 refinement 232.2 against 230.0 ms (four interleaved pairs), after
// split_fused inlined into a one-function split() had taken 235.8 to 232.9 ms.
// ALVRL_SPLIT_NODISPATCH: the one-function split() (split_fused inlined unless
// ALVRL_FUSED_OUTLINE)
#ifndef ALVRL_SPLIT_NODISPATCH
#define ALVRL_SPLIT_DISPATCH
#endif
#if defined(ALVRL_FUSED_OUTLINE) || defined(ALVRL_SPLIT_DISPATCH)
#define ALVRL_FUSED_INL __noinline__
#else
#define ALVRL_FUSED_INL __forceinline__
#endif
// the profile marks inline: split() called them out of line (C4 refinement
// 233.3-234.8 against 234.8-235.1 ms, profiles/r05/inl/); ALVRL_MARK_OUTLINE: calls
#ifdef ALVRL_MARK_OUTLINE
#define ALVRL_MARK_INL
#else
#define ALVRL_MARK_INL __forceinline__
#endif
// developer A/B: split() inlined into its callers (ALVRL_SPLIT_INLINE)
#ifdef ALVRL_SPLIT_INLINE
#define ALVRL_SPLIT_INL __forceinline__
#else
#define ALVRL_SPLIT_INL
#endif
#ifdef ALVRL_POP_INLINE
#define ALVRL_POP_INL __forceinline__
#else
#define ALVRL_POP_INL __noinline__
#endif
using CJ = const ALVRL_AS4 JobDev;
using CC = const ALVRL_AS4 Common;
using CT = const ALVRL_AS4 Team;
template <class T>
__device__ __forceinline__ const ALVRL_AS4 T& uni(const ALVRL_AS4 T& r)
{
    const uint64_t p = (uint64_t)&r;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return *reinterpret_cast<const ALVRL_AS4 T*>(((uint64_t)hi << 32) | lo);
}
// any other reference (a part's view in LDS) as it is: an integer round trip
// would turn it into a generic pointer
template <class T>
__device__ __forceinline__ const T& uni(const T& r) { return r; }
__device__ __forceinline__ void trace(CC& cm, uint32_t phase, uint32_t value)
{
    if (cm.trace && threadIdx.x == 0 && blockIdx.x < 256)
        __hip_atomic_store(&cm.trace[blockIdx.x], ((unsigned long long)phase << 32) | value, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
// A counter add through a typed global pointer: HIP's atomicAdd on a plain
// pointer is a flat atomic, and one flat operation anywhere in a function makes
// the compiler's later waits there wait for every memory operation in flight
// (a flat op may complete out of order with respect to either counter)
__device__ __forceinline__ void gadd(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned long long*)p, v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// Developer event log (tools/evlog.py reads it): compiled in only with
// -DALVRL_EVLOG; thread 0 of a workgroup appends (wall ticks, tag | block,
// a | b).  Timestamps without printf's host round trips.
#ifdef ALVRL_EVLOG
#define EVLOG(cm, tag, a, b) do { if ((cm).evlog && threadIdx.x == 0) {                                        \
        const uint32_t ei_ = __hip_atomic_fetch_add((__attribute__((address_space(1))) uint32_t*)(cm).evlog_n, \
                                                    1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);           \
        if (ei_ < (cm).evlog_cap) {                                                                          \
            auto* e_ = (__attribute__((address_space(1))) unsigned long long*)((cm).evlog + 3ull * ei_);      \
            e_[0] = __builtin_amdgcn_s_memrealtime();                                                        \
            e_[1] = ((unsigned long long)(tag) << 32) | blockIdx.x;                                          \
            e_[2] = ((unsigned long long)(uint32_t)(a) << 32) | (uint32_t)(b);                               \
        } } } while (0)
#else
#define EVLOG(cm, tag, a, b) ((void)0)
#endif
// team counters
enum { TS_ENQ, TS_HSTART, TS_HDONE, TS_COMMIT, TS_STEAL, TS_WAIT_TMO, TS_OWN, TS_IDLE_EXIT, TS_LSIDE,
       TS_HIDLE, TS_RIDLE, TS_HBUSY, TS_RBUSY, TS_ACQ, TS_REL, TS_PSPLIT, TS_PSOLO, TS_POWN, TS_POTHER,
       TS_PWAIT, TS_N };   // *IDLE/*BUSY: wall ticks (100 MHz) summed
__device__ __forceinline__ void tcount(CC& cm, int k)
{
    if (cm.tstat) gadd(&cm.tstat[k], 1ull);
}
__device__ __forceinline__ void tadd(CC& cm, int k, unsigned long long v)
{
    if (cm.tstat) gadd(&cm.tstat[k], v);
}

// Phase timer of lane 0 (s_memtime deltas summed over jobs).
enum { PF_COLW, PF_INIT, PF_UNCL, PF_WSAMP, PF_DIR, PF_PROJ, PF_SORT, PF_CVF, PF_CVR, PF_ARGMIN,
       PF_CTRL, PF_REPS, PF_V_COEF, PF_V_REC, PF_V_RED, PF_P_STAGE, PF_P_COMP, PF_V_OWN, PF_V_CW,
       PF_V_ISSUE, PF_V_DATA, PF_T_HEAP, PF_T_ENQ, PF_T_WAIT, PF_T_SIDE, PF_T_COMMIT, PF_T_SNAP, PF_T_STATE,
       PF_NSPLIT, PF_SPLITCOLS, PF_N };
static const char* kPfNames[PF_N] = {"column weights", "initial clusters", "unclustered var",
                                     "split: centres", "split: direction", "split: projections",
                                     "split: sort", "split: variance fwd", "split: variance rev",
                                     "split: argmin+add", "heap/snapshot/ctrl", "representatives",
                                     // the split engine's coefficient waves (m >= 4096; the
                                     // > 256-row engine adds its own phases to the first three)
                                     " coef wave <=192 rows: chain", " coef wave <=192 rows: (block 3)",
                                     " coef wave <=192 rows: reduce", " coef wave <=192 rows: flush",
                                     " proj: compute",
                                     " coef wave 193-256 rows: chain", " coef wave 193-256 rows: block 3",
                                     " coef wave 193-256 rows: (reduce)", " coef wave 193-256 rows: (flush)",
                                     "ctrl: heap pop/snapshot", "ctrl: enqueue", "ctrl: wait for helper",
                                     "ctrl: side splits", "ctrl: commit", "ctrl: snapshot", "ctrl: state check",
                                     "#splits", "#split columns"};
constexpr int kPfSmall = 2;   // split-phase table of small splits: m < 64, 64 <= m < 256
// (in LDS: a reference to a private Prof made every mark a per-lane flat load
// of p, whose wait also waited out the stores in flight)
struct Prof {
    unsigned long long* p;
    long long t;
    int sm;                      // small-split class of the split in progress (-1: none)
    __device__ ALVRL_MARK_INL void mark(int id);
    __device__ void count(int id, unsigned long long v) { if (p && threadIdx.x == 0) gadd(&p[id], v); }
};
// split-size histogram after the phase totals: per log2(columns) bucket
// (count, split cycles, variance cycles, cycles before the projections)
constexpr int kPfBuckets = 18;
constexpr int kPfWaveBusy = PF_N + 4 * kPfBuckets;   // per-wave busy cycles in the variance passes (+ 8 wall)
constexpr int kPfSmallAt = kPfWaveBusy + 6 * kWaves;   // [NB < 4 | NB == 4][busy, wall, reduce][wave]
constexpr int kPfSmallPh = PF_ARGMIN - PF_WSAMP + 1;
constexpr int kPfTotal = kPfSmallAt + kPfSmall * kPfSmallPh;
__device__ ALVRL_MARK_INL void Prof::mark(int id)
{
    if (p && threadIdx.x == 0) {
        const long long now = clock64();
        gadd(&p[id], (unsigned long long)(now - t));
        if (sm >= 0 && id >= PF_WSAMP && id <= PF_ARGMIN)
            gadd(&p[kPfSmallAt + sm * kPfSmallPh + (id - PF_WSAMP)], (unsigned long long)(now - t));
        t = now;
    }
}
__device__ __forceinline__ int pf_bucket(uint32_t m) { return min(kPfBuckets - 1, 31 - (int)__builtin_clz(max(m, 1u))); }

// Per-column coefficients of the variance recurrence, read as broadcasts.
struct Coef { double w, Wo, a, bb, rw, Wn, rWn; uint32_t vrl, pad; };
struct VarGroup {
    Coef cf[4][kCH];         // coefficients of chunk k in cf[k % 4]
    float res_fu[2 * kCH], res_fi[2 * kCH];   // column sums of the last chunk pair, written out by wave 3
    double Wcur;
    float res_u, res_i;
};

constexpr int kHeapLog = 96;
struct Ctl {
    VarGroup vg[2];
    float tracingVar, unclIntVar, clUnderVar, clIntVar;
    float sh_clUnderVar, sh_clIntVar;
    int heap_n, sh_heap_n, singles_n, sh_singles_n;
    int err;
    uint32_t b, e, vrl1, vrl2, draw_k;
    uint32_t fi1, fi2;       // split_fused: the two centres' positions in the cluster
    int degenerate;
    float diffLen, nd;
    int go, do_snap, stop, refined;
    int tmode, side;
    unsigned long long sw;   // the popped cluster's state word, fetched by pop_wave (team mode)
    // the heap top's state word as enqueue_candidates read it, kept when no
    // helper can change it before the leader's next pop (pre_b: its begin, or ~0)
    unsigned long long pre_sw;
    uint32_t pre_b;
    // the queue tail the leader has written slots up to; published to
    // team.ctl[1] (publish_tail) at the next split_team or stop_team
    uint32_t qtail;        // the queue tail (always current; published at publish_tail)
    int qpend;
    uint32_t qhead;        // a queue head seen earlier (<= the real one: a room bound)
    uint32_t early_b;      // the cluster enqueue_early queued (its heap node is flagged), or ~0
    uint32_t* prec;        // this pop's trace record (ALVRL_POP_TRACE), or null
    // the v3 variance engine over row groups of <= 256 rows (variance_passes):
    // this call's first row, whether it is the first / last group, and the
    // running block-ordered row sums carried between groups (2 passes x m x (u, i))
    uint32_t g_row0;
    int g_first, g_last;
    double* g_carry;
    int team_off;          // the job's team was retired after a timed-out wait (split_team)
    uint32_t yb, ye, j;
    unsigned long long t0;
    float avg;
    // reductions
    float nrm3[3];
    float best_v[kWaves];
    uint32_t best_i[kWaves];
    uint32_t cnt[kWaves];
    uint32_t zeros, lo_or, hi_or, lo_and, hi_and;
    // heap writes since the last snapshot (lane 0)
    uint32_t hlog[kHeapLog];
    int hlog_n, hlog_full;
    int hlds;              // the heap is in the LDS pool (team mode, between splits), else in J.heap
    void* hpool;           // the LDS pool (generic address; accessed through typed LDS pointers only)
};

// ------------------------------------------------------------ helpers --
// Global-address-space view of a pointer: loads through it are global_load
// (vmcnt only).  Through a generic pointer they are flat loads, which also
// count in lgkmcnt -- every LDS wait and every barrier would then wait for
// the prefetches in flight.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gp(const T* p)
{
    return (const __attribute__((address_space(1))) T*)p;
}
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gpw(T* p)
{
    return (__attribute__((address_space(1))) T*)p;
}
// LDS views of pointers that noinline functions receive as generic ones:
// through a generic pointer every access is a flat op, and a flat op makes
// the next LDS wait also wait for every global load in flight (vmcnt(0)).
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef __attribute__((address_space(3))) float lds_f32;
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T* lp(T* p)
{
    return (__attribute__((address_space(3))) T*)p;
}
__device__ __forceinline__ float2 ldg2(const float2* base, size_t i)
{
    const unsigned long long u = gp(reinterpret_cast<const unsigned long long*>(base))[i];
    return make_float2(__uint_as_float((uint32_t)u), __uint_as_float((uint32_t)(u >> 32)));
}

struct RowRef { size_t base, stride; };
__device__ __forceinline__ RowRef row_ref(CJ& J, uint32_t r)
{
    return J.contig ? RowRef{(size_t)(J.off0 + r), (size_t)J.stride0} : RowRef{(size_t)J.roff[r], (size_t)J.rstride[r]};
}
__device__ __forceinline__ float Rmean(CC& cm, RowRef rr, uint32_t v)
{
    return ldg2(cm.Rt, rr.base + (size_t)v * rr.stride).x;
}

// Sequential stream of one (stage, cluster range) (see oracle smp_t).
struct Smp {
    uint32_t seed, pass, a, b, c, k, blk;
    U4 buf;
    __device__ void init(uint32_t s, uint32_t p, uint32_t a_, uint32_t b_, uint32_t c_)
    {
        seed = s; pass = p; a = a_; b = b_; c = c_; k = 0; blk = 0xFFFFFFFFu;
    }
    __device__ float next()
    {
        const uint32_t bl = k >> 2;
        if (bl != blk) { buf = philox4x32_10(a, b, bl, (kDomCluster << 24) | (c & 0xFFFFFFu), seed, pass); blk = bl; }
        const uint32_t s = k & 3;
        const uint32_t x = s == 0 ? buf.x : (s == 1 ? buf.y : (s == 2 ? buf.z : buf.w));
        ++k;
        return u01(x);
    }
};

__device__ __forceinline__ float draw_at(uint32_t seed, uint32_t pass, uint32_t a, uint32_t b,
                                         uint32_t c, uint32_t k)
{
    const U4 r = philox4x32_10(a, b, k >> 2, (kDomCluster << 24) | (c & 0xFFFFFFu), seed, pass);
    const uint32_t s = k & 3;
    return u01(s == 0 ? r.x : (s == 1 ? r.y : (s == 2 ? r.z : r.w)));
}

// weightedSample (Preprocessor.cpp:1534-1580) by one whole wave, in the
// blocked summation order of the oracle (alvrl_preproc.c weighted_sample):
// a block of 64 weights per step, Hillis-Steele within rows of 16 (DPP
// row_shr 1/2/4/8), row bases b1 = t0, b2 = b1 + t1, b3 = b2 + t2, block
// bases S_{b+1} = S_b + total_b, and the pick is the first index whose
// prefix S_b + P[l] reaches alpha (a ballot).  Weights come from wv[i], or
// colw[ids[i]] when wv is null; index zero_at weighs 0 (the second centre of
// split(), drawn with colw[vrl1] = 0).  Every lane returns the same index;
// *prob = w / weightSum as in the reference.
template <int K>
__device__ __forceinline__ float row_shr_masked(float x, uint32_t lane)
{
    const float v = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x110 + K, 0xF, 0xF, false));
    return (lane & 15u) >= (uint32_t)K ? v : 0.0f;
}
__device__ __forceinline__ float ws_block_wave(float x, uint32_t lane, float* tot)
{
    x = x + row_shr_masked<1>(x, lane);
    x = x + row_shr_masked<2>(x, lane);
    x = x + row_shr_masked<4>(x, lane);
    x = x + row_shr_masked<8>(x, lane);
    const float t0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 15));
    const float t1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 31));
    const float t2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 47));
    const float t3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
    const float b1 = t0, b2 = b1 + t1, b3 = b2 + t2;
    *tot = b3 + t3;
    const uint32_t r = lane >> 4;
    const float base = r == 0 ? 0.0f : (r == 1 ? b1 : (r == 2 ? b2 : b3));
    return base + x;
}
// The stream state comes by value and its new draw count goes back with the
// pick (a reference to the caller's private Smp made every draw a per-lane
// flat load and store); the caller resumes the stream at WsPick::k.
struct WsPick { uint32_t idx, k; int err; float prob; };
__device__ ALVRL_WS_INL WsPick weighted_sample_wave(const float* wv, const float* colw, const uint32_t* ids,
                                                    uint32_t m, Smp smp, uint32_t zero_at, bool want_prob,
                                                    bool wv_lds = false)
{
    const uint32_t lane = threadIdx.x & 63;
    WsPick r{0u, smp.k, 0, 1.0f};
    if (m == 0) { r.err = 1; return r; }
    if (m == 1) return r;
    auto ld = [&](uint32_t i) -> float {
        const uint32_t c = min(i, m - 1);
        const float x = wv ? (wv_lds ? lp(wv)[c] : gp(wv)[c]) : gp(colw)[gp(ids)[c]];
        return (i >= m || i == zero_at) ? 0.0f : x;
    };
    const uint32_t nb = (m + 63) / 64;
    float weightSum = 0.0f;
    float cur = ld(lane);
    for (uint32_t b = 0; b < nb; b++) {
        const float nxt = b + 1 < nb ? ld((b + 1) * 64 + lane) : 0.0f;
        float tot;
        (void)ws_block_wave(cur, lane, &tot);
        weightSum = weightSum + tot;
        cur = nxt;
    }
    uint32_t idx = 0;
    if (weightSum <= 0) {
        int tries = 0;
        do {
            idx = (uint32_t)((float)0u + smp.next() * (float)m);
            if (++tries > 1000) { r.err = 1; idx = 0; break; }
        } while (idx >= m);
        if (want_prob) r.prob = (float)(1.0 / (double)m);
    } else {
        const float alpha = smp.next() * weightSum;
        float S = 0.0f;
        cur = ld(lane);
        for (uint32_t b = 0; b < nb; b++) {
            const float nxt = b + 1 < nb ? ld((b + 1) * 64 + lane) : 0.0f;
            float tot;
            const float P = ws_block_wave(cur, lane, &tot);
            const unsigned long long hit = __ballot(b * 64 + lane < m && S + P >= alpha);
            if (hit) { idx = b * 64 + (uint32_t)__ffsll((long long)hit) - 1; break; }
            S = S + tot;
            cur = nxt;
        }
        if (want_prob) {
            const float wi = idx == zero_at ? 0.0f : (wv ? (wv_lds ? lp(wv)[idx] : gp(wv)[idx]) : gp(colw)[gp(ids)[idx]]);
            r.prob = wi / weightSum;
        }
    }
    r.idx = idx;
    r.k = smp.k;
    return r;
}

// weighted_sample_wave's pick, bit for bit, with the whole workgroup: every
// wave forms the block totals of its blocks (the same DPP tree), 8 blocks'
// weights in flight per lane, into tot[] (LDS, nb floats); lane 0 then runs
// the two sequential float chains: weightSum = sum of the totals in block
// order, and the search S_b = S_{b-1} + tot_{b-1} for the first block with
// S_b + tot_b >= alpha.  That test is the wave's per-lane test of that block:
// the prefixes P[l] grow with l (non-negative weights, monotone rounding),
// a lane past m or at zero_at adds +0.0, and the block's last prefix is its
// total (b3 + t3 either way), so some lane of block b reaches alpha exactly
// when S_b + tot_b does.  Wave 0 then scans that block alone.  Every thread
// returns the pick; the caller resumes the stream at WsPick::k.
__device__ __noinline__ WsPick weighted_sample_wg(const float* wv, bool wv_lds, uint32_t m, Smp smp, uint32_t zero_at,
                                                  float* tot_in)
{
    const int tid = threadIdx.x;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = (uint32_t)(tid & 63);
    auto* const tot = lp(tot_in);
    __shared__ uint32_t res[3];
    m = (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
    wv_lds = __builtin_amdgcn_readfirstlane((int)wv_lds) != 0;
    WsPick r{0u, smp.k, 0, 1.0f};
    if (m <= 1) { r.err = m == 0; return r; }
    auto ld = [&](uint32_t i) -> float {
        const uint32_t c = min(i, m - 1);
        const float x = wv_lds ? lp(wv)[c] : gp(wv)[c];
        return (i >= m || i == zero_at) ? 0.0f : x;
    };
    const uint32_t nb = (m + 63) / 64;
    constexpr uint32_t B = 8;
    for (uint32_t b0 = wave; b0 < nb; b0 += B * kWaves) {
        float x[B];
#pragma unroll
        for (uint32_t j = 0; j < B; j++) x[j] = ld(min(b0 + j * kWaves, nb - 1) * 64 + lane);
#pragma unroll
        for (uint32_t j = 0; j < B; j++) {
            float t;
            (void)ws_block_wave(x[j], lane, &t);
            if (lane == 0 && b0 + j * kWaves < nb) tot[b0 + j * kWaves] = t;
        }
    }
    __syncthreads();
    if (wave == 0) {
        // the chains take 64 totals per LDS read, one v_readlane each
        auto rl = [](float v, int j) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j)); };
        float weightSum = 0.0f;
        for (uint32_t g0 = 0; g0 < nb; g0 += 64) {
            const float v = tot[min(g0 + lane, nb - 1)];
            if (g0 + 64 <= nb) {
#pragma unroll
                for (int j = 0; j < 64; j++) weightSum = weightSum + rl(v, j);
            } else {
                for (uint32_t j = 0; j < nb - g0; j++) weightSum = weightSum + rl(v, (int)j);
            }
        }
        uint32_t idx = 0;
        int err = 0;
        if (weightSum <= 0) {
            int tries = 0;
            do {
                idx = (uint32_t)((float)0u + smp.next() * (float)m);
                if (++tries > 1000) { err = 1; idx = 0; break; }
            } while (idx >= m);
        } else {
            const float alpha = smp.next() * weightSum;
            float S = 0.0f;
            uint32_t bh = nb;
            for (uint32_t g0 = 0; g0 < nb && bh == nb; g0 += 64) {
                const float v = tot[min(g0 + lane, nb - 1)];
                const uint32_t n = min(64u, nb - g0);
                for (uint32_t j = 0; j < n; j++) {
                    const float t = rl(v, (int)j);
                    if (S + t >= alpha) { bh = g0 + j; break; }
                    S = S + t;
                }
            }
            if (bh < nb) {
                float t;
                const float P = ws_block_wave(ld(bh * 64 + lane), lane, &t);
                const unsigned long long hit = __ballot(bh * 64 + lane < m && S + P >= alpha);
                if (hit) idx = bh * 64 + (uint32_t)__ffsll((long long)hit) - 1;
            }
        }
        if (lane == 0) { res[0] = idx; res[1] = smp.k; res[2] = (uint32_t)err; }
    }
    __syncthreads();
    r.idx = res[0]; r.k = res[1]; r.err = (int)res[2];
    __syncthreads();
    return r;
}

// deterministic Box-Muller x (oracle alvrl_o_det_std_normal_x)
__device__ double det_log(double x)
{
    int e = 0;
    while (x < 0.70710678118654752440) { x = x * 2.0; e--; }
    const double z = (x - 1.0) / (x + 1.0), z2 = z * z;
    double term = z, sum = 0.0;
    for (int k = 1; k <= 41; k += 2) { sum = sum + term / (double)k; term = term * z2; }
    return 2.0 * sum + (double)e * 0.69314718055994530942;
}
__device__ double det_cos(double phi)
{
    const double PI_ = 3.14159265358979323846;
    double x = phi;
    if (x > PI_) x = 2.0 * PI_ - x;
    double sign = 1.0;
    if (x > 0.5 * PI_) { x = PI_ - x; sign = -1.0; }
    const double x2 = x * x;
    double term = 1.0, sum = 0.0;
    for (int k = 0; k < 14; k++) { sum = sum + term; term = -term * x2 / (double)((2 * k + 1) * (2 * k + 2)); }
    return sign * sum;
}
__device__ float det_std_normal_x(float sx, float sy)
{
    const double r = sqrt(-2.0 * det_log(1.0 - (double)sx));
    const double phi = 2.0 * 3.14159265358979323846 * (double)sy;
    return (float)(det_cos(phi) * r);
}

// LDS-pool bounds checks (build with -DALVRL_LDS_CHECK, tools/build_variant.sh):
// an index past the pool is counted in g_lds_viol, reported once with printf,
// and the access is skipped (a typed ds_* access past the allocation would be
// dropped or read 0 silently; a flat one faults).  alvrl_refine fails with
// ALVRL_ERR_NUMERIC when any was seen.  Off in the product build.
#ifdef ALVRL_LDS_CHECK
__device__ unsigned int g_lds_viol;
#define LDS_OK(cond, what, a, b)                                                                          \
    ((cond) ? true                                                                                       \
            : ((atomicAdd(&g_lds_viol, 1u) == 0u                                                         \
                    ? (void)printf("ALVRL_LDS_CHECK %s: %ld %ld (block %d thread %d)\n", what, (long)(a),  \
                                   (long)(b), (int)blockIdx.x, (int)threadIdx.x)                         \
                    : (void)0),                                                                          \
               false))
#else
#define LDS_OK(cond, what, a, b) true
#endif

// ------------------------------------------------------------- heap --
__device__ __forceinline__ bool cless(const CNode& a, const CNode& b)
{
    return a.uvar + a.ivar < b.uvar + b.ivar;
}
// The heap is worked by lane 0 (pops by wave 0).  It lives in J.heap, and in
// team mode the leader keeps it in the LDS pool between splits (heap_move):
// each pop's sift-down is a chain of dependent heap reads, and at N >= 4 GPUs
// the leader's pops are the refinement's critical path.  Accesses are typed
// LDS or typed global ones on a uniform branch (HeapRef), never flat: flat
// accesses to LDS faulted on this platform (memory aperture violation).
// Every write is logged so a snapshot copies only what changed.
typedef uint32_t hnode_v __attribute__((ext_vector_type(4)));
constexpr int kHeapLdsMax = (int)(kPoolBytes / sizeof(hnode_v));
typedef __attribute__((address_space(1))) hnode_v* hnode_p;
typedef __attribute__((address_space(3))) hnode_v* hnode_l;
__device__ __forceinline__ hnode_p hnodes(CNode* p) { return (hnode_p)p; }
struct HeapRef {
    hnode_p g;
    hnode_l l;
    int lds;
    __device__ __forceinline__ hnode_v ld(long i) const
    {
        if (lds) {
            if (!LDS_OK(i >= 0 && i < kHeapLdsMax, "heap load", i, kHeapLdsMax)) return hnode_v{0u, 0u, 0u, 0u};
            return l[i];
        }
        return g[i];
    }
    __device__ __forceinline__ void st(long i, hnode_v v) const
    {
        if (lds) {
            if (LDS_OK(i >= 0 && i < kHeapLdsMax, "heap store", i, kHeapLdsMax)) l[i] = v;
        } else {
            g[i] = v;
        }
    }
    // the placement known at compile time (L == lds): an LDS heap's accesses
    // then wait on LDS counters only, not on the memory loads in flight
    template <bool L>
    __device__ __forceinline__ hnode_v ldt(long i) const
    {
        if (L) {
            if (!LDS_OK(i >= 0 && i < kHeapLdsMax, "heap load", i, kHeapLdsMax)) return hnode_v{0u, 0u, 0u, 0u};
            return l[i];
        }
        return g[i];
    }
    template <bool L>
    __device__ __forceinline__ void stt(long i, hnode_v v) const
    {
        if (L) {
            if (LDS_OK(i >= 0 && i < kHeapLdsMax, "heap store", i, kHeapLdsMax)) l[i] = v;
        } else {
            g[i] = v;
        }
    }
};
__device__ __forceinline__ CNode hld(hnode_p H, long i)
{
    const hnode_v v = H[i];
    return CNode{__uint_as_float(v.x), __uint_as_float(v.y), v.z, v.w};
}
// PL: the heap's placement, -1 = H.lds at run time, 0 = global, 1 = LDS
template <int PL = -1>
__device__ __forceinline__ CNode hld(const HeapRef& H, long i)
{
    hnode_v v;
    if constexpr (PL < 0) v = H.ld(i);
    else v = H.template ldt<PL == 1>(i);
    return CNode{__uint_as_float(v.x), __uint_as_float(v.y), v.z, v.w};
}
template <int PL = -1>
__device__ __forceinline__ void hst(const HeapRef& H, long i, const CNode& c)
{
    const hnode_v v{__float_as_uint(c.uvar), __float_as_uint(c.ivar), c.begin, c.end};
    if constexpr (PL < 0) H.st(i, v);
    else H.template stt<PL == 1>(i, v);
}
__device__ __forceinline__ void heap_log(Ctl& C, long i)
{
    if (C.hlog_n < kHeapLog) C.hlog[C.hlog_n++] = (uint32_t)i;
    else C.hlog_full = 1;
}
template <int PL = -1>
__device__ void push_heap_(const HeapRef& first, long hole, long top, CNode value, Ctl& C)
{
    long parent = (hole - 1) / 2;
    while (hole > top) {
        const CNode pn = hld<PL>(first, parent);
        if (!cless(pn, value)) break;
        hst<PL>(first, hole, pn);
        heap_log(C, hole);
        hole = parent;
        parent = (hole - 1) / 2;
    }
    hst<PL>(first, hole, value);
    heap_log(C, hole);
}

__device__ __forceinline__ HeapRef heap_of(CJ& J, const Ctl& C)
{
    return HeapRef{hnodes(J.heap), lp(reinterpret_cast<hnode_v*>(C.hpool)), C.hlds};
}
// lane-0-only Clustering::addCluster (:549-579)
// (a single's id is read from J.vrls, or with an agent-scope load from spec:
// a commit's range copy into J.vrls may still be in flight)
template <int PL = -1>
__device__ void add_cluster(CJ& J_in, Ctl& C, uint32_t begin, uint32_t end, float uvar, float ivar,
                            const uint32_t* spec = nullptr, uint32_t flags = 0u, uint32_t single_id = ~0u)
{
    CJ& J = uni(J_in);
    if (end == begin) { C.err = 1; return; }
    if (end == begin + 1) {
        gpw(J.singles)[C.singles_n++] =
            single_id != ~0u ? single_id
            : spec ? __hip_atomic_load(&gp(spec)[begin], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : gp(J.vrls)[begin];
        if (uvar != 0) C.err = 1;
        C.clIntVar += ivar;
    } else {
        CNode cn{uvar, ivar, begin, end | flags | (spec ? kEndS : 0u)};
        const HeapRef H = heap_of(J, C);
        hst<PL>(H, C.heap_n++, cn);
        heap_log(C, C.heap_n - 1);
        push_heap_<PL>(H, C.heap_n - 1, 0, cn, C);
        C.clUnderVar += uvar;
        C.clIntVar += ivar;
    }
}
// std::pop_heap (Clustering's heap pop, via pop_multi's move of the top to
// the end and __adjust_heap + __push_heap), on wave 0.  The sift-down path is
// found five levels per round trip: lane t loads node t of the 62-node
// subtree below the current hole, each lane decides whether it is the child
// __adjust_heap would descend to (the right one unless right < left; the left
// one when it is the only child), and the path is read off the ballot.  The
// moved last element then climbs that path while the node above it is less
// (__push_heap), which only needs the path's original values: lane i holds
// path node i.  Final array = std::pop_heap's; the slots written are logged.
// With state set (team mode), lane 0 also fetches the popped cluster's state
// word while the sift-down runs (split_team's first look): C.sw.
#ifdef ALVRL_PT_POP   // diagnostic: trace points 1-3 inside the pop, 4 after its barrier
#define PT_POP(k) do { if ((threadIdx.x & 63) == 0 && C.prec) gpw(C.prec)[k] = (uint32_t)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define PT_POP(k) do { } while (0)
#endif
template <bool LH>
__device__ __forceinline__ CNode pop_wave_t(CJ& J, Ctl& C, const unsigned long long* state)
{
    const int lane = (int)(threadIdx.x & 63);
    const HeapRef H = heap_of(J, C);
    auto hld = [&](const HeapRef& Hr, long i) {
        const hnode_v v = Hr.ldt<LH>(i);
        return CNode{__uint_as_float(v.x), __uint_as_float(v.y), v.z, v.w};
    };
    auto hst = [&](const HeapRef& Hr, long i, const CNode& c) {
        Hr.stt<LH>(i, hnode_v{__float_as_uint(c.uvar), __float_as_uint(c.ivar), c.begin, c.end});
    };
    const long n = __builtin_amdgcn_readfirstlane(C.heap_n);
    const CNode top = hld(H, 0);
    unsigned long long sw = 0;
    PT_POP(1);
    // a node this leader never queued: no helper is on it (kStNone)
    if (state && lane == 0 && (top.end & kEndQ))
        sw = __hip_atomic_load(&gp(state)[top.begin], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (n > 1) {
        const long len = n - 1;
        const CNode value = hld(H, len);
        const float vkey = value.uvar + value.ivar;
        long h = 0;                        // current path node (uniform)
        int L = 0;                         // path length: p_0 = 0 .. p_L
        long pidx = 0;                     // lane i: index of path node i
        hnode_v pv = {0u, 0u, 0u, 0u};     // lane i: its original value
        const int k = 31 - __builtin_clz((uint32_t)lane + 2);
        const long j = (long)lane + 2 - (1l << k);
        bool more = true;
        while (more) {
            const long idx = ((h + 1) << k) - 1 + j;
            const bool ex = lane < 62 && idx < len;
            hnode_v v = {0u, 0u, 0u, 0u};
            if (ex) v = H.ldt<LH>(idx);
            const float key = __uint_as_float(v.x) + __uint_as_float(v.y);
            // the sibling's key and existence: a DPP quad permutation [1,0,3,2]
            // (siblings are lanes 2i, 2i + 1), not an LDS round trip
            const float skey = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(key), 0xB1, 0xF, 0xF, false));
            const int sex = __builtin_amdgcn_mov_dpp((int)ex, 0xB1, 0xF, 0xF, false);
            // left (even j): taken unless the right exists and !(right < left)
            const bool chosen = (j & 1) ? (ex && !(key < skey)) : (ex && (!sex || skey < key));
            const unsigned long long mask = __ballot(chosen);
            long jp = 0;
            for (int kk = 1; kk <= 5; kk++) {
                const int lc = (1 << kk) - 2 + 2 * (int)jp;
                const unsigned long long two = (mask >> lc) & 3ull;
                if (!two) { more = false; break; }
                const int c = (two & 1ull) ? lc : lc + 1;
                jp = 2 * jp + (c - lc);
                const long ic = ((h + 1) << kk) - 1 + jp;
                L++;
                if constexpr (LH) {
                    // an LDS heap: the path's values are read back below
                    if (lane == L) pidx = ic;
                } else {
                    hnode_v vc;
                    vc.x = __builtin_amdgcn_readlane(v.x, c);
                    vc.y = __builtin_amdgcn_readlane(v.y, c);
                    vc.z = __builtin_amdgcn_readlane(v.z, c);
                    vc.w = __builtin_amdgcn_readlane(v.w, c);
                    if (lane == L) { pidx = ic; pv = vc; }
                }
                if (kk == 5) h = ic;
            }
        }
        // (nothing is written during the search: lane i reads path node i)
        if (LH && lane >= 1 && lane <= L) pv = H.ldt<LH>(pidx);
        PT_POP(2);
        // __push_heap from p_L: climbs while the node above is less
        const bool stay = lane >= 1 && lane <= L && !((__uint_as_float(pv.x) + __uint_as_float(pv.y)) < vkey);
        const unsigned long long nf = __ballot(stay);
        const int fin = nf ? 63 - __builtin_clzll(nf) : 0;
        hnode_v up;
        up.x = __shfl_down(pv.x, 1); up.y = __shfl_down(pv.y, 1);
        up.z = __shfl_down(pv.z, 1); up.w = __shfl_down(pv.w, 1);
        if (lane < fin) H.stt<LH>(pidx, up);
        if (lane == fin) hst(H, pidx, value);
        if (lane == 0) hst(H, len, top);
        const int base = C.hlog_n, w = fin + 2;
        if (base + w <= kHeapLog) {
            if (lane <= fin) C.hlog[base + lane] = (uint32_t)pidx;
            if (lane == 0) { C.hlog[base + fin + 1] = (uint32_t)len; C.hlog_n = base + w; }
        } else if (lane == 0) {
            C.hlog_full = 1;
        }
    }
    if (lane == 0) {
        C.heap_n = (int)n - 1;
        C.clUnderVar -= top.uvar;
        C.clIntVar -= top.ivar;
        if (state) C.sw = sw;
        C.pre_b = ~0u;
    }
    PT_POP(3);
    return CNode{top.uvar, top.ivar, top.begin, top.end & kEndMask};
}
__device__ ALVRL_POP_INL CNode pop_wave(CJ& J_in, Ctl& C, const unsigned long long* state = nullptr)
{
    CJ& J = uni(J_in);
    return C.hlds ? pop_wave_t<true>(J, C, state) : pop_wave_t<false>(J, C, state);
}

__device__ __forceinline__ uint32_t n_clusters(const Ctl& C) { return (uint32_t)(C.singles_n + C.heap_n); }
__device__ __forceinline__ float unclustered_var(const Ctl& C) { return C.tracingVar + C.unclIntVar; }
__device__ __forceinline__ float clustered_var(const Ctl& C) { return C.tracingVar + C.clUnderVar + C.clIntVar; }
__device__ float conv_const(Ctl& C, uint32_t nvrl, float pu)
{
    const float c = ((float)nvrl * pu + (float)n_clusters(C)) * clustered_var(C);
    if (!isfinite(c) || c <= 0) C.err = 1;
    return c;
}
__device__ float lower_bound(Ctl& C, uint32_t nvrl, float pu)
{
    const float c = ((float)nvrl * pu + (float)n_clusters(C)) * unclustered_var(C);
    if (!isfinite(c) || c <= 0) C.err = 1;
    return c;
}

// collective snapshot / restore (:686-699)
// Between two snapshots the singles only grow and the heap changes where the
// log says; a snapshot copies those (or everything after a restore or a log
// overflow).  The snapshot's content is the same as a full copy.
__device__ void snapshot(CJ& J_in, Ctl& C)
{
    CJ& J = uni(J_in);
    const int nh = C.heap_n, ns = C.singles_n;
    const HeapRef H = heap_of(J, C);
    const hnode_p SH = hnodes(J.sh_heap);
    if (C.hlog_full) {
        for (int i = threadIdx.x; i < nh; i += kThreads) SH[i] = H.ld(i);
        for (int i = threadIdx.x; i < ns; i += kThreads) gpw(J.sh_singles)[i] = gp(J.singles)[i];
    } else {
        const int nl = C.hlog_n;
        for (int t = threadIdx.x; t < nl; t += kThreads) {
            const uint32_t i = C.hlog[t];
            if ((int)i < nh) SH[i] = H.ld(i);
        }
        for (int i = C.sh_singles_n + threadIdx.x; i < ns; i += kThreads) gpw(J.sh_singles)[i] = gp(J.singles)[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        C.sh_clUnderVar = C.clUnderVar; C.sh_clIntVar = C.clIntVar;
        C.sh_heap_n = nh; C.sh_singles_n = ns;
        C.hlog_n = 0; C.hlog_full = 0;
    }
    __syncthreads();
}
__device__ void restore(CJ& J_in, Ctl& C)
{
    CJ& J = uni(J_in);
    // The singles below the snapshot's count never change (appends only), and
    // the heap differs from the snapshot only where the log says.
    const int nh = C.sh_heap_n, ns = C.sh_singles_n;
    const HeapRef H = heap_of(J, C);
    const hnode_p SH = hnodes(J.sh_heap);
    if (C.hlog_full) {
        for (int i = threadIdx.x; i < nh; i += kThreads) H.st(i, SH[i]);
        for (int i = threadIdx.x; i < ns; i += kThreads) gpw(J.singles)[i] = gp(J.sh_singles)[i];
    } else {
        const int nl = C.hlog_n;
        for (int t = threadIdx.x; t < nl; t += kThreads) {
            const uint32_t i = C.hlog[t];
            if ((int)i < nh) H.st(i, SH[i]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        C.clUnderVar = C.sh_clUnderVar; C.clIntVar = C.sh_clIntVar;
        C.heap_n = nh; C.singles_n = ns;
        C.hlog_n = 0; C.hlog_full = 0;
    }
    __syncthreads();
}

// Collective: move the heap into the LDS pool (to_lds, if it fits with room
// for one more split's net growth) or back to J.heap.  The pool is the split
// engines' scratch, so the heap goes back before any split by this workgroup
// and before the representatives.  Content and order are unchanged.
__device__ void heap_move(CJ& J_in, Ctl& C, bool to_lds)
{
    CJ& J = uni(J_in);
    __syncthreads();
    const int n = C.heap_n;
    const bool cur = C.hlds != 0;
    if (to_lds ? (cur || n + 2 > kHeapLdsMax) : !cur) return;   // uniform
    const hnode_p G = hnodes(J.heap);
    const hnode_l L = lp(reinterpret_cast<hnode_v*>(C.hpool));
    if (!LDS_OK(n <= kHeapLdsMax, "heap_move", n, kHeapLdsMax)) return;
    for (int i = threadIdx.x; i < n; i += kThreads) {
        if (to_lds) L[i] = G[i];
        else G[i] = L[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) C.hlds = to_lds ? 1 : 0;
    __syncthreads();
}

// ------------------------------------------------ variance recurrence --

__device__ __forceinline__ double readlane_d(double v, uint32_t l)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Lane l receives lane l+off's value (used only where l < off): permlane
// swaps for the cross-row steps, DPP row shifts inside a 16-lane row -- VALU
// only, no LDS round trip.
template <int OFF>
__device__ __forceinline__ uint32_t from_lane_plus(uint32_t v)
{
    if constexpr (OFF == 32) return __builtin_amdgcn_permlane32_swap(v, v, false, false)[1];
    else if constexpr (OFF == 16) return __builtin_amdgcn_permlane16_swap(v, v, false, false)[1];
    else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x100 + OFF, 0xF, 0xF, false);
}
template <int OFF>
__device__ __forceinline__ double from_lane_plus_d(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const uint32_t lo = from_lane_plus<OFF>((uint32_t)u), hi = from_lane_plus<OFF>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int OFF>
__device__ __forceinline__ float from_lane_plus_f(float v) { return __uint_as_float(from_lane_plus<OFF>(__float_as_uint(v))); }

// The row-reduction order shared with the oracle (wsum_d / wsum_f): lane l
// holds the in-order sum of rows l, l+64, ...; the halving tree p[l] +=
// p[l+off], off = 32..1, leaves the total in lane 0 (lanes >= off compute
// values nothing reads).  N independent sums are combined level by level.
template <int N>
__device__ __forceinline__ void tree_dn(double* p)
{
#define ALVRL_TREE_LEVEL(OFF) { double o[N]; _Pragma("unroll") for (int q = 0; q < N; q++) o[q] = from_lane_plus_d<OFF>(p[q]); \
                                _Pragma("unroll") for (int q = 0; q < N; q++) p[q] = p[q] + o[q]; }
    ALVRL_TREE_LEVEL(32) ALVRL_TREE_LEVEL(16) ALVRL_TREE_LEVEL(8) ALVRL_TREE_LEVEL(4) ALVRL_TREE_LEVEL(2) ALVRL_TREE_LEVEL(1)
#undef ALVRL_TREE_LEVEL
}
template <int N>
__device__ __forceinline__ void tree_fn(float* p)
{
#define ALVRL_TREE_LEVEL(OFF) { float o[N]; _Pragma("unroll") for (int q = 0; q < N; q++) o[q] = from_lane_plus_f<OFF>(p[q]); \
                                _Pragma("unroll") for (int q = 0; q < N; q++) p[q] = p[q] + o[q]; }
    ALVRL_TREE_LEVEL(32) ALVRL_TREE_LEVEL(16) ALVRL_TREE_LEVEL(8) ALVRL_TREE_LEVEL(4) ALVRL_TREE_LEVEL(2) ALVRL_TREE_LEVEL(1)
#undef ALVRL_TREE_LEVEL
}
__device__ __forceinline__ double tree_d(double p) { tree_dn<1>(&p); return p; }
__device__ __forceinline__ float tree_f(float p) { tree_fn<1>(&p); return p; }

// Per-column coefficients of the recurrence for one chunk (one lane each),
// the running weight total in the reference's sequential order via
// v_readlane.  Runs on one full wave; kw = this lane's (weight bits << 32 |
// vrl) of the chunk (lanes >= cn ignored).
__device__ __forceinline__ void chunk_coefs(VarGroup& V, Ctl& C, unsigned long long kw, uint32_t cn, Coef* out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t vrl = (uint32_t)kw;
    const double w = lane < cn ? (double)__uint_as_float((uint32_t)(kw >> 32)) : 1.0;
    if (lane < cn && (!isfinite(w) || w <= 0)) C.err = 1;
    double W = V.Wcur, Wo = 0.0, Wn = 0.0;
    for (uint32_t c = 0; c < cn; c++) {
        const double wc = readlane_d(w, c);
        if (lane == c) Wo = W;
        W = W + wc;
        if (lane == c) Wn = W;
    }
    if (lane < cn) {
        Coef k;
        k.w = w; k.Wo = Wo; k.Wn = Wn;
        k.a = (Wn * Wn) / (Wo * Wo);
        k.rw = 1.0 / w;
        k.bb = (k.rw + 1.0 / Wo);
        k.rWn = 1.0 / Wn;
        k.vrl = vrl; k.pad = 0;
        out[lane] = k;
    }
    if (lane == 0) V.Wcur = W;
}

// calculateClusterVariance (:1058-1120), one or two passes at once: pass g
// (g = 0 forward over base[0..m), g = 1 backward) runs on the 4 waves
// [4g, 4g+4).  Rows are split in 64-row blocks, block b on wave b mod 4 of
// the pass (lane = row mod 64).  Chunks of kCH columns are software
// pipelined:
//  phase 1 (every chunk)  wave 3 forms the coefficients of chunk k+3 (ring of
//           4; its (vrl, weight) was loaded a chunk earlier) and writes the
//           last pair's column sums out; the row waves issue the entries of
//           chunk k+2 (register ring of 3, ids from the LDS coefficients) and
//           run the recurrence of chunk k, writing each row's prefix terms
//           locw*(M/W) and locw*(V*W) to T[k & 1][c][block][lane];
//  phase 2 (every 2nd chunk)  the pass's 4 waves reduce the pair's columns
//           in the shared row order (in-order over the blocks per lane, then
//           the lane tree), all of a wave's sums interleaved.
// No global store and no dependent global load sits on the row waves'
// critical path.  With FU == false only the final variances are formed.
template <bool TLDS, bool FU>
__device__ __noinline__ void variance_passes_t(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* base,
                                               uint32_t m, int npass, float* fu0, float* fi0, float* fu1, float* fi1,
                                               unsigned char* pool, Prof* pf)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const uint32_t R = J.nrows;
    const uint32_t NB = (R + 63) / 64;
    const int tid = threadIdx.x;
    const int g = tid / kGT, lt = tid - g * kGT, w = lt >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const bool active = g < npass;
    float* fu = g == 0 ? fu0 : fu1;
    float* fi = g == 0 ? fi0 : fi1;
    VarGroup& V = C.vg[g];
    double* st = J.st + (size_t)g * 3 * R;
    const size_t tsz = (size_t)kCH * NB * 64;          // one chunk's terms
    double2* T = TLDS ? reinterpret_cast<double2*>(pool) + (size_t)g * 2 * tsz
                      : reinterpret_cast<double2*>(J.bufM) + (size_t)g * 2 * tsz;
    unsigned long long* cw = J.keys1;
    long long t0 = pf ? (long long)clock64() : 0, t1 = 0, tc = 0, trc = 0, trd = 0;
    const uint32_t nch = (m + kCH - 1) / kCH;
    auto cn_of = [&](uint32_t k) { return min((uint32_t)kCH, m - k * kCH); };
    auto kw_of = [&](uint32_t k) -> unsigned long long {   // this lane's (weight, vrl) of chunk k
        if (k >= nch) return 0ull;
        const uint32_t i = k * kCH + min(lane, cn_of(k) - 1);
        return gp(cw)[g == 0 ? i : m - 1 - i];
    };

    // (vrl, weight) of every column of the cluster, gathered in parallel once
    {
        constexpr int B = 8;
        for (uint32_t i0 = (uint32_t)tid; i0 < m; i0 += B * kThreads) {
            uint32_t v[B];
#pragma unroll
            for (int b = 0; b < B; b++) v[b] = gp(base)[min(i0 + (uint32_t)b * kThreads, m - 1)];
            float wv[B];
#pragma unroll
            for (int b = 0; b < B; b++) wv[b] = gp(J.colw)[v[b]];
#pragma unroll
            for (int b = 0; b < B; b++)
                if (i0 + (uint32_t)b * kThreads < m)
                    cw[i0 + (uint32_t)b * kThreads] = ((unsigned long long)__float_as_uint(wv[b]) << 32) | v[b];
        }
    }
    if (active && lt == 0) V.Wcur = 0.0;
    __syncthreads();
    unsigned long long kw_next = 0;                 // wave 3: (weight, vrl) of the next coefficient chunk
    if (active && w == 3) {
        for (uint32_t k = 0; k < 3 && k < nch; k++) chunk_coefs(V, C, kw_of(k), cn_of(k), V.cf[k]);
        kw_next = kw_of(3);
    }
    __syncthreads();

    // the first block of this wave lives in registers across chunks
    const uint32_t b0 = (uint32_t)w;
    const bool own = active && b0 < NB && b0 * 64 + lane < R;
    const uint32_t r0 = b0 * 64 + lane;
    const RowRef rr0 = own ? row_ref(J, r0) : RowRef{0, 0};
    const double lw0 = own ? J.locw[r0] : 0.0;
    double sum0 = 0.0, M0 = 0.0, V0 = 0.0;
    float2 bufA[kCH], bufB[kCH], bufC[kCH];
    auto load_chunk = [&](uint32_t k, float2* dst) {    // ids from the LDS coefficients of chunk k
        const Coef* cf = V.cf[k % 4];
        const uint32_t cn = cn_of(k);
#pragma unroll
#ifdef ALVRL_EXP_NOLOAD
        for (int c = 0; c < kCH; c++) dst[c] = make_float2((float)cf[(uint32_t)c < cn ? c : 0].vrl * 1e-7f + rr0.base * 1e-9f, 0.25f);
#else
        for (int c = 0; c < kCH; c++) dst[c] = ldg2(cm.Rt, rr0.base + (size_t)cf[(uint32_t)c < cn ? c : 0].vrl * rr0.stride);
#endif
    };
    if (own) { load_chunk(0, bufA); if (nch > 1) load_chunk(1, bufB); }
    if (active && NB > 4)
        for (uint32_t b = b0 + 4; b < NB; b += 4)
            if (b * 64 + lane < R) { const uint32_t r = b * 64 + lane; st[r] = 0.0; st[R + r] = 0.0; st[2 * R + r] = 0.0; }
    if (pf) { t1 = clock64(); tc += t1 - t0; t0 = t1; }

    constexpr int NQ = kCH / 4;                      // columns per wave per chunk in phase 2
    // phase 1 of chunk k: entries in cur, chunk k+2's into pre
    const bool wprof = cm.prof != nullptr;
    long long wbusy = 0, wred = 0, wwall0 = wprof ? (long long)clock64() : 0;
    auto step = [&](uint32_t k, float2* cur, float2* pre) {
        const long long ws0 = wprof ? (long long)clock64() : 0;
        const uint32_t c0 = k * kCH, cn = cn_of(k);
        const Coef* cf = V.cf[k % 4];
        double2* Tk = T + (size_t)(k & 1) * tsz;
        if (FU && active && w == 3 && k >= 2 && (k & 1) == 0 && lane < 2u * kCH) {
            // the pair (k-2, k-1) was reduced after chunk k-1: write it out
            const uint32_t j = lane / kCH, c = lane % kCH, kk = k - 2 + j;
            if (c < cn_of(kk)) { const uint32_t n = kk * kCH + c; fu[n] = V.res_fu[lane]; fi[n] = V.res_fi[lane]; }
        }
        if (active && w == 3 && k + 3 < nch) {
            chunk_coefs(V, C, kw_next, cn_of(k + 3), V.cf[(k + 3) % 4]);
            kw_next = kw_of(k + 4);
        }
        if (own) {
            if (k + 2 < nch) load_chunk(k + 2, pre);      // in flight during the next two chunks
            if (cn == (uint32_t)kCH && k > 0) {            // full chunk, no first column: no guards
                Coef qn = cf[0];
#pragma unroll
                for (int c = 0; c < kCH; c++) {
                    const Coef q = qn;
                    if (c + 1 < kCH) qn = cf[c + 1];
                    const double x = (double)cur[c].x;
                    const double tmp = q.w * sum0 - q.Wo * x;
                    M0 = q.a * M0 + q.bb * (tmp * tmp);
                    V0 = V0 + (double)cur[c].y * q.rw;
                    sum0 = sum0 + x;
                    if (FU) Tk[((size_t)c * NB + b0) * 64 + lane] = make_double2(lw0 * (M0 * q.rWn), lw0 * (V0 * q.Wn));
                }
            } else {
#pragma unroll
                for (int c = 0; c < kCH; c++) {
                    if ((uint32_t)c < cn) {
                        const Coef q = cf[c];
                        const double x = (double)cur[c].x;
                        const double tmp = q.w * sum0 - q.Wo * x;
                        if (c0 + c > 0) M0 = q.a * M0 + q.bb * (tmp * tmp);
                        V0 = V0 + (double)cur[c].y * q.rw;
                        sum0 = sum0 + x;
                        if (FU) Tk[((size_t)c * NB + b0) * 64 + lane] = make_double2(lw0 * (M0 * q.rWn), lw0 * (V0 * q.Wn));
                    }
                }
            }
        }
        if (active && NB > 4) {
            for (uint32_t b = b0 + 4; b < NB; b += 4) {
                if (b * 64 + lane >= R) continue;
                const uint32_t r = b * 64 + lane;
                const RowRef rr = row_ref(J, r);
                const double lw = J.locw[r];
                float2 e[kCH];
#pragma unroll
                for (int c = 0; c < kCH; c++) e[c] = ldg2(cm.Rt, rr.base + (size_t)cf[(uint32_t)c < cn ? c : 0].vrl * rr.stride);
                double sum = st[r], M = st[R + r], Vs = st[2 * R + r];
#pragma unroll
                for (int c = 0; c < kCH; c++) {
                    if ((uint32_t)c < cn) {
                        const Coef q = cf[c];
                        const double x = (double)e[c].x;
                        const double tmp = q.w * sum - q.Wo * x;
                        if (c0 + c > 0) M = q.a * M + q.bb * (tmp * tmp);
                        Vs = Vs + (double)e[c].y * q.rw;
                        sum = sum + x;
                        if (FU) Tk[((size_t)c * NB + b) * 64 + lane] = make_double2(lw * (M * q.rWn), lw * (Vs * q.Wn));
                    }
                }
                st[r] = sum; st[R + r] = M; st[2 * R + r] = Vs;
            }
        }
        if (wprof) wbusy += (long long)clock64() - ws0;
        __syncthreads();
        if (pf) { t1 = clock64(); trc += t1 - t0; t0 = t1; }
    };
    // phase 2: reduce chunks kf .. kf+nk-1 (nk <= 2) into the staging sums
    auto reduce = [&](uint32_t kf, uint32_t nk) {
        const long long ws0 = wprof ? (long long)clock64() : 0;
        if (active) {
            // per 64-row block the halving tree (rows past R as +0.0), the
            // block totals added in block order (oracle wsum_blk)
            double pz[4 * NQ];                       // [pu of 2*NQ columns, pi of 2*NQ columns]
            for (uint32_t b = 0; b < NB; b++) {
                double tz[4 * NQ];
#pragma unroll
                for (int j = 0; j < 2; j++) {
#pragma unroll
                    for (int q = 0; q < NQ; q++) {
                        const uint32_t c = (uint32_t)w + 4u * q;
                        double pu = 0.0, pi = 0.0;
                        if ((uint32_t)j < nk && c < cn_of(kf + j) && b * 64 + lane < R) {
                            const double2 t = (T + (size_t)((kf + j) & 1) * tsz)[((size_t)c * NB + b) * 64 + lane];
                            pu = t.x; pi = t.y;
                        }
                        tz[j * NQ + q] = pu;
                        tz[2 * NQ + j * NQ + q] = pi;
                    }
                }
                tree_dn<4 * NQ>(tz);
#pragma unroll
                for (int i = 0; i < 4 * NQ; i++) pz[i] = b == 0 ? tz[i] : pz[i] + tz[i];
            }
            if (lane == 0) {
#pragma unroll
                for (int j = 0; j < 2; j++) {
#pragma unroll
                    for (int q = 0; q < NQ; q++) {
                        const uint32_t c = (uint32_t)w + 4u * q;
                        if ((uint32_t)j < nk && c < cn_of(kf + j)) {
                            const uint32_t slot = (uint32_t)j * kCH + c;
                            V.res_fi[slot] = (float)pz[2 * NQ + j * NQ + q];
                            V.res_fu[slot] = (kf + j) * kCH + c == 0 ? 0.0f : (float)pz[j * NQ + q];
                        }
                    }
                }
            }
        }
        if (wprof) wred += (long long)clock64() - ws0;
        __syncthreads();
        if (pf) { t1 = clock64(); trd += t1 - t0; t0 = t1; }
    };
    static_assert(kCH % 4 == 0, "phase 2: 4 waves x kCH/4 columns per chunk");
    auto after = [&](uint32_t k) { if (FU && (k & 1)) reduce(k - 1, 2); };
    for (uint32_t k = 0; k < nch; k += 3) {
        step(k, bufA, bufC); after(k);
        if (k + 1 < nch) { step(k + 1, bufB, bufA); after(k + 1); }
        if (k + 2 < nch) { step(k + 2, bufC, bufB); after(k + 2); }
    }
    if (FU && (nch & 1)) reduce(nch - 1, 1);
    if (wprof && lane == 0 && m >= 4096) {
        gadd(&cm.prof[kPfWaveBusy + tid / 64], (unsigned long long)wbusy);
        gadd(&cm.prof[kPfWaveBusy + kWaves + tid / 64], (unsigned long long)((long long)clock64() - wwall0));
        gadd(&cm.prof[kPfWaveBusy + 2 * kWaves + tid / 64], (unsigned long long)wred);
    }
    // the last pair's sums, the final variances
    if (FU && active && w == 3 && nch > 0 && lane < 2u * kCH) {
        const uint32_t kf = (nch & 1) ? nch - 1 : nch - 2;
        const uint32_t j = lane / kCH, c = lane % kCH, kk = kf + j;
        if (kk < nch && c < cn_of(kk)) { const uint32_t n = kk * kCH + c; fu[n] = V.res_fu[lane]; fi[n] = V.res_fi[lane]; }
    }
    if (own) { st[r0] = sum0; st[R + r0] = M0; st[2 * R + r0] = V0; }
    __syncthreads();
    if (active && w == 0) {
        if (FU) {
            if (lane == 0) { V.res_u = fu[m - 1]; V.res_i = fi[m - 1]; }
        } else {
            const double Wt = V.Wcur, rW = 1.0 / Wt;
            double pu = 0.0, pi = 0.0;
            for (uint32_t r = lane; r < R; r += 64) {
                pu = pu + J.locw[r] * (st[R + r] * rW);
                pi = pi + J.locw[r] * (st[2 * R + r] * Wt);
            }
            pu = tree_d(pu);
            pi = tree_d(pi);
            if (lane == 0) { V.res_u = (float)pu; V.res_i = (float)pi; }
        }
        if (lane == 0) {
            if (!isfinite(V.res_u) || V.res_u < 0) C.err = 1;
            if (!isfinite(V.res_i) || V.res_i < 0) C.err = 1;
        }
    }
    __syncthreads();
    if (pf) { pf->count(PF_V_COEF, tc); pf->count(PF_V_REC, trc); pf->count(PF_V_RED, trd); }
}


// ---------------------------------------------- split variance engine --
// The two calculateClusterVariance passes of a split (forward over base[0..m)
// and backward, with per-prefix outputs), for local matrices of <= 3 row
// blocks.  Same arithmetic, same operation order and the same row-reduction
// order as variance_passes_t; what changes is the schedule:
//  * each pass has 3 row waves (block b, lane = row mod 64) and one
//    coefficient wave (pass 0: wave 3, pass 1: wave 4, so that the f64 work
//    spreads over the four SIMDs);
//  * one barrier per chunk: during chunk k the row waves run the recurrence
//    of chunk k (T[k & 1]) and issue the entries of chunk k+2, while the
//    coefficient wave reduces chunk k-1 (T[(k-1) & 1]) and forms the
//    coefficients of chunk k+3;
//  * coefficients are stored per chunk as SoA (two columns of one
//    coefficient per ds_read_b128);
//  * the 16 row sums of a chunk (pu, pi of 8 columns) are reduced with a
//    transposed halving tree: at every level the pairs p[l] + p[l+off] of
//    the shared tree are formed for two sums at once, the second in the lanes
//    the tree leaves idle (permlane32/16 swaps, DPP row rotations), so the
//    additions and their operand order are exactly those of tree_dn.
// Coefficients of 64 consecutive columns (8 chunks) of one pass, SoA so a row
// wave reads two columns' worth of one coefficient with one ds_read_b128.
constexpr int kCB64 = 64;
struct CoefBlock { double w[kCB64], Wo[kCB64], a[kCB64], bb[kCB64], rw[kCB64], Wn[kCB64], rWn[kCB64]; uint32_t vrl[kCB64]; };
constexpr uint32_t kSplitTBytes = 2u * 2u * kCH * 4u * 64u * sizeof(double2);     // [pass][k & 1][c][block][lane]
constexpr uint32_t kSplitStageBytes = 2u * 2u * 2u * kCB64 * sizeof(float);      // [pass][block & 1][u|i][64]
constexpr uint32_t kSplitPoolBytes = kSplitTBytes + 2u * 2u * sizeof(CoefBlock) + kSplitStageBytes;
static_assert(kSplitPoolBytes <= kPoolBytes, "split variance engine: pool");

__device__ __forceinline__ double dbl_of(uint32_t hi, uint32_t lo)
{
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ uint32_t lo_of(double d) { return (uint32_t)(unsigned long long)__double_as_longlong(d); }
__device__ __forceinline__ uint32_t hi_of(double d) { return (uint32_t)((unsigned long long)__double_as_longlong(d) >> 32); }
// lanes 0-31: A[l] + A[l+32]; lanes 32-63: B[l-32] + B[l]
__device__ __forceinline__ double swap32_add(double A, double B)
{
    const auto lo = __builtin_amdgcn_permlane32_swap(lo_of(A), lo_of(B), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(hi_of(A), hi_of(B), false, false);
    return dbl_of(hi[0], lo[0]) + dbl_of(hi[1], lo[1]);
}
// per 32 lanes: row 0: A[l] + A[l+16]; row 1: B[l-16] + B[l]
__device__ __forceinline__ double swap16_add(double A, double B)
{
    const auto lo = __builtin_amdgcn_permlane16_swap(lo_of(A), lo_of(B), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(hi_of(A), hi_of(B), false, false);
    return dbl_of(hi[0], lo[0]) + dbl_of(hi[1], lo[1]);
}
// per 16 lanes: lanes 0-7: P[l] + P[l+8]; lanes 8-15: Q[l-8] + Q[l]
__device__ __forceinline__ double pair8_add(double P, double Q, uint32_t lane)
{
    const bool lo = (lane & 8) == 0;
    const double X = lo ? P : Q, Y = lo ? Q : P;
    const uint32_t zl = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo_of(Y), 0x128, 0xF, 0xF, false);   // row_ror:8
    const uint32_t zh = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi_of(Y), 0x128, 0xF, 0xF, false);
    return X + dbl_of(zh, zl);
}
// per 8 lanes: lanes 0-3: P[l] + P[l+4]; lanes 4-7: Q[l-4] + Q[l]
__device__ __forceinline__ double pair4_add(double P, double Q, uint32_t lane)
{
    const bool lo = (lane & 4) == 0;
    const double X = lo ? P : Q, Y = lo ? Q : P;
    const uint32_t al = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo_of(Y), 0x104, 0xF, 0xF, false);   // row_shl:4
    const uint32_t ah = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi_of(Y), 0x104, 0xF, 0xF, false);
    const uint32_t bl = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo_of(Y), 0x114, 0xF, 0xF, false);   // row_shr:4
    const uint32_t bh = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi_of(Y), 0x114, 0xF, 0xF, false);
    return X + (lo ? dbl_of(ah, al) : dbl_of(bh, bl));
}
// v[2c + h] (c < 8: column, h: 0 = pu, 1 = pi) -> the shared-order total of
// value (c, h) in lane 32h + 16(c & 1) + 8((c >> 1) & 1) + 4(c >> 2)
__device__ __forceinline__ double tree16_transposed(const double* v, uint32_t lane)
{
    double u[8], x[4], y[2];
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = swap32_add(v[2 * i], v[2 * i + 1]);
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = swap16_add(u[2 * i], u[2 * i + 1]);
#pragma unroll
    for (int i = 0; i < 2; i++) y[i] = pair8_add(x[2 * i], x[2 * i + 1], lane);
    double z = pair4_add(y[0], y[1], lane);
    z = z + from_lane_plus_d<2>(z);
    z = z + from_lane_plus_d<1>(z);
    return z;
}

// v[2c + h] (c < 4) -> the shared-order total of value (c, h) in lane
// 32h + 16(c & 1) + 8(c >> 1): the same pairs p[l] + p[l+off] as tree_dn
// (an IEEE add is commutative, so which lane holds which operand is free)
__device__ __forceinline__ double tree8_transposed(const double* v, uint32_t lane)
{
    double u[4], x[2];
#pragma unroll
    for (int i = 0; i < 4; i++) u[i] = swap32_add(v[2 * i], v[2 * i + 1]);
#pragma unroll
    for (int i = 0; i < 2; i++) x[i] = swap16_add(u[2 * i], u[2 * i + 1]);
    double z = pair8_add(x[0], x[1], lane);
    z = z + from_lane_plus_d<4>(z);
    z = z + from_lane_plus_d<2>(z);
    z = z + from_lane_plus_d<1>(z);
    return z;
}

// The coefficient wave's share of chunk_coefs for 8 columns of a 64-column
// block: the running total W in the reference's order (v_readlane), the
// column's lane (8j + c) keeping W before (Wo) and after (Wn) its weight.
__device__ __forceinline__ void coef_chain8(double& W, double w, uint32_t j, uint32_t ncol, double& Wo, double& Wn)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c0 = 8 * j;
    if (c0 >= ncol) return;                            // wave-uniform
    // the 8 weights to SGPRs first (independent of W), then the dependent
    // chain of adds; the column's lane keeps W before / after by selects
    double wc[kCH];
#pragma unroll
    for (int c = 0; c < kCH; c++) wc[c] = readlane_d(w, c0 + (uint32_t)c);
    if (ncol - c0 >= (uint32_t)kCH) {
#pragma unroll
        for (int c = 0; c < kCH; c++) {
            const bool me = lane == c0 + (uint32_t)c;
            Wo = me ? W : Wo;
            W = W + wc[c];
            Wn = me ? W : Wn;
        }
    } else {
        const uint32_t n = ncol - c0;
#pragma unroll
        for (int c = 0; c < kCH; c++) {
            if ((uint32_t)c < n) {
                const bool me = lane == c0 + (uint32_t)c;
                Wo = me ? W : Wo;
                W = W + wc[c];
                Wn = me ? W : Wn;
            }
        }
    }
}
// chunk_coefs' divisions for the block's columns, one lane each
__device__ __forceinline__ void coef_block_finish(Ctl& C, double w, double Wo, double Wn, uint32_t vrl, uint32_t ncol,
                                                  CoefBlock* out)
{
    const uint32_t lane = threadIdx.x & 63;
    if (lane < ncol) {
        if (!isfinite(w) || w <= 0) C.err = 1;
        out->w[lane] = w; out->Wo[lane] = Wo; out->Wn[lane] = Wn;
        out->a[lane] = (Wn * Wn) / (Wo * Wo);
        const double rw = 1.0 / w;
        out->rw[lane] = rw;
        out->bb[lane] = (rw + 1.0 / Wo);
        out->rWn[lane] = 1.0 / Wn;
        (void)vrl;
    }
}

// FU == false: only the final variances of npass passes (no prefix terms, no
// reduction per chunk): the rows' final states go to J.st and one wave per
// pass forms the two sums, as variance_passes_t does.
template <bool FU, bool GRP = false>
__device__ __noinline__ void variance_split_v3(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* base,
                                               uint32_t m, int npass, float* fu0, float* fi0, float* fu1, float* fi1,
                                               unsigned char* pool)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    // a group of <= 256 rows (row0 .. row0 + R) of the job's Rfull: the
    // coefficients are the same for every group, the block-ordered row sums
    // continue from the previous group's (C.g_carry), and the prefix results
    // are written by the last group only
    // (GRP = false: one group of all the rows, the constants fold away)
    const uint32_t Rfull = J.nrows, row0 = GRP ? C.g_row0 : 0u;
    const uint32_t R = GRP ? min(Rfull - row0, 256u) : Rfull;
    const bool gfirst = GRP ? C.g_first != 0 : true, glast = GRP ? C.g_last != 0 : true;
    double* const carry = GRP ? C.g_carry : nullptr;
    const uint32_t NB = (R + 63) / 64;                 // <= 4 (block 3 on the coefficient wave)
    const int tid = threadIdx.x, wv = tid >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const int g = wv < 4 ? 0 : 1;
    const bool active = g < npass;
    const bool coefw = active && wv == (g == 0 ? 3 : 4);
    const uint32_t b0 = g == 0 ? (uint32_t)wv : (uint32_t)(wv - 5);      // row block (row waves)
    float* fu = g == 0 ? fu0 : fu1;
    float* fi = g == 0 ? fi0 : fi1;
    VarGroup& V = C.vg[g];
    // per chunk and row block the 16 block totals (pu, pi of 8 columns) of
    // the rows' prefix terms, [k & 1][block][2c + h]
    double* Q = reinterpret_cast<double*>(pool) + (size_t)g * 2 * 4 * 16;
    CoefBlock* ring = reinterpret_cast<CoefBlock*>(pool + kSplitTBytes) + g * 2;
    // prefix results of the last two 64-column blocks, stored out once per
    // block: a global store in every chunk would make the next chunk's LDS
    // reads wait for it (vmcnt(0) for the store's registers)
    float* stg = reinterpret_cast<float*>(pool + kSplitTBytes + 4 * sizeof(CoefBlock)) + g * 2 * 2 * kCB64;
    unsigned long long* cw = J.keys1;
    const uint32_t nch = (m + kCH - 1) / kCH;
    const uint32_t nblk = (m + kCB64 - 1) / kCB64;
    auto cn_of = [&](uint32_t k) { return min((uint32_t)kCH, m - k * kCH); };
    auto ncol_of = [&](uint32_t b) { return min((uint32_t)kCB64, m - b * kCB64); };
    // profile counters: 32-bit per-wave sums (a split's chunk steps add up to
    // well under 2^32 ticks), added to cm.prof once at the end; 64-bit ones
    // cost VGPRs of the budget, and a global atomic per step would put its
    // round trip in front of every barrier
    const bool wprof = cm.prof != nullptr && m >= 4096;
    const int pbase = kPfWaveBusy + (NB == 4 ? 3 * kWaves : 0);
    auto padd = [&](int idx, long long v) {
        if (lane == 0) gadd(&cm.prof[idx], (unsigned long long)v);
    };
    uint32_t pc_busy = 0, pc_red = 0, pc_sp[4] = {0, 0, 0, 0};
    const long long wall0 = wprof ? (long long)clock64() : 0;

    // (vrl, weight) of every column of the cluster, gathered in parallel once
    {
        constexpr int B = 8;
        for (uint32_t i0 = (uint32_t)tid; i0 < m; i0 += B * kThreads) {
            uint32_t v[B];
#pragma unroll
            for (int b = 0; b < B; b++) v[b] = gp(base)[min(i0 + (uint32_t)b * kThreads, m - 1)];
            float wt[B];
#pragma unroll
            for (int b = 0; b < B; b++) wt[b] = gp(J.colw)[v[b]];
#pragma unroll
            for (int b = 0; b < B; b++)
                if (i0 + (uint32_t)b * kThreads < m)
                    cw[i0 + (uint32_t)b * kThreads] = ((unsigned long long)__float_as_uint(wt[b]) << 32) | v[b];
        }
    }
    __syncthreads();
    // coefficient wave state: this lane's column of the block being formed
    const auto cwp = gp(cw);
    auto kw_of_blk = [&](uint32_t b) -> unsigned long long {
        if (b >= nblk) return 0ull;
        const uint32_t i = b * kCB64 + min(lane, ncol_of(b) - 1);
        return cwp[g == 0 ? i : m - 1 - i];
    };
    double W = 0.0, cWo = 0.0, cWn = 0.0, cw_w = 1.0;
    uint32_t cw_v = 0;
    unsigned long long kwN = 0;
    auto take = [&](unsigned long long kw, uint32_t b) {   // start forming block b
        cw_v = (uint32_t)kw;
        cw_w = lane < ncol_of(b) ? (double)__uint_as_float((uint32_t)(kw >> 32)) : 1.0;
        cWo = 0.0; cWn = 0.0;
        if (lane < ncol_of(b)) ring[b & 1].vrl[lane] = cw_v;
    };
    if (coefw) {
        take(kw_of_blk(0), 0);
        for (uint32_t j = 0; j < 8; j++) coef_chain8(W, cw_w, j, ncol_of(0), cWo, cWn);
        coef_block_finish(C, cw_w, cWo, cWn, cw_v, ncol_of(0), &ring[0]);
        kwN = kw_of_blk(1);
    }
    __syncthreads();

    const bool roww = active && !coefw && b0 < NB;
    // every lane of a row wave runs the recurrence (rows past R on row R-1's
    // data: their terms are never reduced), so no load or store is predicated
    const uint32_t r0 = min(b0 * 64 + lane, R - 1);
    const RowRef rr0 = roww ? row_ref(J, row0 + r0) : RowRef{0, 0};
    // rows past R carry weight 0: their prefix terms are +0.0 exactly (M, V >= 0),
    // which is what the reduction order wants from them (no per-term select)
    const double lw0 = roww && b0 * 64 + lane < R ? J.locw[row0 + r0] : 0.0;

    // coefficient wave: the 16 row sums of chunk kk, the row blocks' tree
    // totals added in block order (wsum_blk), one sum per lane 0-15
    auto reduce = [&](uint32_t kk) {
        const uint32_t cn = cn_of(kk);
        const double* Qk = Q + (size_t)(kk & 1) * 4 * 16;
        const uint32_t sl = lane & 15, c = sl >> 1, h = sl & 1;
        const uint32_t n = kk * kCH + c;
        double* const cy = carry + ((size_t)g * m + min(n, m - 1)) * 2 + h;   // this pass's running sum
        double acc = gfirst ? Qk[sl] : gp(cy)[0];
#pragma unroll
        for (uint32_t b = gfirst ? 1 : 0; b < 4; b++)
            if (b < NB) acc = acc + Qk[b * 16 + sl];
        if (!glast) {
            if (lane < 16 && c < cn) gpw(cy)[0] = acc;
            return;
        }
        if (lane < 16 && c < cn) {
            const float f = h == 0 ? (n == 0 ? 0.0f : (float)acc) : (float)acc;
            stg[(((kk / 8) & 1) * 2 + h) * kCB64 + (kk % 8) * kCH + c] = f;
            if (n == m - 1) {
                if (h == 0) V.res_u = f; else V.res_i = f;
                if (!isfinite(f) || f < 0) C.err = 1;
            }
        }
    };

    auto flush = [&](uint32_t b) {                     // block b's prefix results, one column per lane
        const uint32_t col = b * kCB64 + lane;
        if (glast && col < m) {                                 // global, not flat: a flat store would make
            gpw(fu)[col] = stg[((b & 1) * 2 + 0) * kCB64 + lane];   // every LDS wait a vmcnt(0)
            gpw(fi)[col] = stg[((b & 1) * 2 + 1) * kCB64 + lane];
        }
    };
    // the recurrence of chunk k for one 64-row block (lane = row); each half
    // chunk's 8 prefix terms (pu, pi of 4 columns) are reduced over the block
    // as soon as they exist (tree8_transposed) and their totals go to Q[k & 1][blk].
    // Register budget: the engine is called once per split, and every
    // callee-saved VGPR it touches is saved and restored per call (207 KB
    // per workgroup at 101 registers).  So the coefficients
    // arrive one column ahead (not the whole chunk's 7 x 8 doubles up
    // front), and only half a chunk's terms are live at once.
    auto rec = [&](uint32_t k, const float2* cur, uint32_t blk, double lw, double& sum0, double& M0, double& V0) {
        const uint32_t c0 = k * kCH, cn = cn_of(k);
        const CoefBlock& q = ring[(k / 8) & 1];
        const uint32_t o = (k % 8) * kCH;
        double th[kCH];                                // half a chunk's prefix terms (pu, pi) per column
        auto half_done = [&](uint32_t hsel) {          // the block's halving tree (rows past R enter as +0.0)
            if (!FU) return;
#ifdef ALVRL_EXP_NOTREE
            const double z = th[0] + th[3] + th[6];   // timing experiment: no reduction
#else
            const double z = tree8_transposed(th, lane);
#endif
            if ((lane & 7) == 0) {
                const uint32_t h = lane >> 5, c = 4 * hsel + 2 * ((lane >> 3) & 1) + ((lane >> 4) & 1);
                Q[((size_t)(k & 1) * 4 + blk) * 16 + 2 * c + h] = z;
            }
        };
        if (cn == (uint32_t)kCH && k > 0) {            // full chunk, no first column: no guards
            struct CCol { double w, Wo, a, bb, rw, Wn, rWn; };
            auto ldc = [&](int c) {                    // one column's coefficients (LDS broadcasts)
                return CCol{q.w[o + c], q.Wo[o + c], q.a[o + c], q.bb[o + c], q.rw[o + c], q.Wn[o + c], q.rWn[o + c]};
            };
            auto col = [&](const CCol& k2, float2 e, double* t) {
                const double x = (double)e.x;
                const double tmp = k2.w * sum0 - k2.Wo * x;
                M0 = k2.a * M0 + k2.bb * (tmp * tmp);
                V0 = V0 + (double)e.y * k2.rw;
                sum0 = sum0 + x;
                if (FU) { t[0] = lw * (M0 * k2.rWn); t[1] = lw * (V0 * k2.Wn); }
            };
            // coefficients two columns ahead (one ahead: 0.3-1 % slower, profiles/r03/engine/pf2/)
            CCol k0 = ldc(0), k1 = ldc(1), k2 = k1;
#pragma unroll
            for (int c = 0; c < kCH; c++) {
                if (c + 2 < kCH) k2 = ldc(c + 2);
                col(k0, cur[c], &th[2 * (c & 3)]);
                k0 = k1; k1 = k2;
                if (c == 3) half_done(0);
            }
            half_done(1);
        } else {
#pragma unroll
            for (int c = 0; c < kCH; c++) {
                double* t = &th[2 * (c & 3)];
                if ((uint32_t)c < cn) {
                    const double x = (double)cur[c].x;
                    const double tmp = q.w[o + c] * sum0 - q.Wo[o + c] * x;
                    if (c0 + c > 0) M0 = q.a[o + c] * M0 + q.bb[o + c] * (tmp * tmp);
                    V0 = V0 + (double)cur[c].y * q.rw[o + c];
                    sum0 = sum0 + x;
                    if (FU) { t[0] = lw * (M0 * q.rWn[o + c]); t[1] = lw * (V0 * q.Wn[o + c]); }
                } else if (FU) {
                    t[0] = 0.0; t[1] = 0.0;
                }
                if (c == 3) half_done(0);
                if (c == 7) half_done(1);
            }
        }
    };
    // entries of chunk k for a row block (ids from the LDS ring)
    auto load_rows = [&](const float2* Rt, size_t rstride, uint32_t k, float2* dst) {
        const uint32_t* ids = &ring[(k / 8) & 1].vrl[(k % 8) * kCH];
        const uint32_t cn = cn_of(k);
#ifdef ALVRL_EXP_NOLOAD
#pragma unroll
        for (int c = 0; c < kCH; c++) dst[c] = make_float2((float)ids[(uint32_t)c < cn ? c : 0] * 1e-7f + (float)lane * 1e-9f, 0.25f);
#elif defined(ALVRL_EXP_NOBAR)
        // timing experiment without the chunk barriers: ids may be stale, keep them in range
#pragma unroll
        for (int c = 0; c < kCH; c++) dst[c] = ldg2(Rt, (size_t)min(ids[(uint32_t)c < cn ? c : 0], cm.nvrl - 1) * rstride);
#else
#pragma unroll
        for (int c = 0; c < kCH; c++) dst[c] = ldg2(Rt, (size_t)ids[(uint32_t)c < cn ? c : 0] * rstride);
#endif
    };

    if (coefw) {
        // chunk k = 8B + j: reduce chunk k-1; form block B+1's coefficients
        // (8 columns of the running total per chunk, the divisions at j = 7);
        // with 4 row blocks this wave also runs block 3's recurrence (its
        // entries one chunk ahead, ping-pong buffers).  Block B+2's (weight,
        // vrl) is loaded at j = 0 and taken 8 chunks later (one block per
        // outer iteration: no register copy of a load in flight)
        const bool own3 = NB == 4;
        const uint32_t r3 = min(3u * 64u + lane, R - 1);
        const RowRef rr3 = own3 ? row_ref(J, row0 + r3) : RowRef{0, 0};
        const double lw3 = own3 && 3u * 64u + lane < R ? J.locw[row0 + r3] : 0.0;
        const float2* const Rt3 = cm.Rt + rr3.base;
        const size_t rs3 = rr3.stride;
        double sum3 = 0.0, M3 = 0.0, V3 = 0.0;
        float2 cA[kCH], cB[kCH];
        if (own3) load_rows(Rt3, rs3, 0, cA);
        auto stepc = [&](uint32_t B, uint32_t j, uint32_t nb, float2* cur, float2* nxt) {
            const uint32_t k = B * 8 + j;
            const long long ws0 = wprof ? (long long)clock64() : 0;
#ifndef ALVRL_EXP_NORED
            if (FU && !own3 && k >= 1) reduce(k - 1);
#endif
            const long long ws1 = wprof ? (long long)clock64() : 0;
            if (FU && !own3 && j == 0 && B >= 1) flush(B - 1);
            const long long ws2 = wprof ? (long long)clock64() : 0;
            if (nb < nblk) {
#ifdef ALVRL_EXP_NOCHAIN
                // timing experiment (results invalid): no running weight total
                cWo = 1.0 + (double)(nb * 64u + lane); cWn = cWo + 1.0;   // telescoping like the real totals
#else
                coef_chain8(W, cw_w, j, ncol_of(nb), cWo, cWn);
#endif
                if (j == 7 || k == nch - 1) coef_block_finish(C, cw_w, cWo, cWn, cw_v, ncol_of(nb), &ring[nb & 1]);
            }
            const long long ws3 = wprof ? (long long)clock64() : 0;
            if (own3) {
                load_rows(Rt3, rs3, min(k + 1, nch - 1), nxt);
                rec(k, cur, 3, lw3, sum3, M3, V3);
            }
            if (wprof) {   // sub-phases: reduce, flush, chain, rec 3
                const long long ws4 = (long long)clock64();
                pc_red += (uint32_t)(ws4 - ws0);
#ifndef ALVRL_EXP_STAMP
                pc_sp[0] += (uint32_t)(ws1 - ws0); pc_sp[1] += (uint32_t)(ws2 - ws1);
                pc_sp[2] += (uint32_t)(ws3 - ws2); pc_sp[3] += (uint32_t)(ws4 - ws3);
#endif
            }
            #ifndef ALVRL_EXP_NOBAR
            __syncthreads();
            #endif
        };
#ifdef ALVRL_EXP_COEFPRIO
        __builtin_amdgcn_s_setprio(ALVRL_EXP_COEFPRIO);
#endif
        for (uint32_t B = 0; B * 8 < nch; B++) {
            const uint32_t nb = B + 1;
            if (nb < nblk) take(kwN, nb);
            kwN = kw_of_blk(nb + 1);
#pragma unroll 1
            for (uint32_t j = 0; j < 8; j += 2) {
                if (B * 8 + j >= nch) break;
                stepc(B, j, nb, cA, cB);
                if (B * 8 + j + 1 >= nch) break;
                stepc(B, j + 1, nb, cB, cA);
            }
        }
#ifdef ALVRL_EXP_COEFPRIO
        __builtin_amdgcn_s_setprio(0);
#endif
        if (FU) {
            if (!own3) {
                reduce(nch - 1);
                flush((nch - 1) / 8);
            }
        } else {
            if (lane == 0) V.Wcur = W;
            if (own3 && 3u * 64u + lane < R) {
                double* st = J.st + (size_t)g * 3 * Rfull;
                gpw(st)[Rfull + row0 + 3u * 64u + lane] = M3;
                gpw(st)[2 * Rfull + row0 + 3u * 64u + lane] = V3;
            }
        }
    } else if (roww) {
        double sum0 = 0.0, M0 = 0.0, V0 = 0.0;
        float2 bufA[kCH], bufB[kCH], bufC[kCH];
        // a register copy: cm is reached through a generic pointer, and a flat
        // reload after every barrier would wait for every load in flight
        const float2* const Rt = cm.Rt + rr0.base;
        const size_t rstride = rr0.stride;
        auto load_chunk = [&](uint32_t k, float2* dst) { load_rows(Rt, rstride, k, dst); };
        load_chunk(0, bufA);
        load_chunk(min(1u, nch - 1), bufB);
        // chunk k: issue the entries of chunk k+2 (clamped: the last chunk is
        // re-read, so the wait for chunk k is always "all but the 16 youngest"),
        // run the recurrence of chunk k into T[k & 1]
        // with 4 row blocks the coefficient wave also runs block 3, and the
        // row wave of block 0 takes the chunk reductions and block flushes
        const bool red = FU && NB == 4 && b0 == 0;
        auto step = [&](uint32_t k, float2* cur, float2* pre) {
            const long long ws0 = wprof ? (long long)clock64() : 0;
#ifdef ALVRL_EXP_STAMP
            // developer timing (profile builds): load issue, recurrence, barrier wait
            auto stamp = []() {
                unsigned long long t;
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
                __builtin_amdgcn_sched_barrier(0);
                return t;
            };
            const unsigned long long s0 = stamp();
#endif
            load_chunk(min(k + 2, nch - 1), pre);
#ifdef ALVRL_EXP_STAMP
            const unsigned long long s1 = stamp();
#endif
            if (red) {
                if (k >= 1) reduce(k - 1);
                if ((k & 7) == 0 && k >= 8) flush(k / 8 - 1);
            }
            rec(k, cur, b0, lw0, sum0, M0, V0);
            if (wprof) pc_busy += (uint32_t)((long long)clock64() - ws0);
#ifdef ALVRL_EXP_STAMP
            const unsigned long long s2 = stamp();
#endif
            #ifndef ALVRL_EXP_NOBAR
            __syncthreads();
            #endif
#ifdef ALVRL_EXP_STAMP
            const unsigned long long s3 = stamp();
            if (wprof) { pc_sp[0] += (uint32_t)(s1 - s0); pc_sp[1] += (uint32_t)(s2 - s1); pc_sp[2] += (uint32_t)(s3 - s2); }
#endif
        };
        for (uint32_t k = 0; k < nch; k += 3) {
            step(k, bufA, bufC);
            if (k + 1 < nch) step(k + 1, bufB, bufA);
            if (k + 2 < nch) step(k + 2, bufC, bufB);
        }
            if (red) {
            reduce(nch - 1);
            flush((nch - 1) / 8);
        }
        if (!FU && b0 * 64 + lane < R) {
            double* st = J.st + (size_t)g * 3 * Rfull;
            gpw(st)[Rfull + row0 + b0 * 64 + lane] = M0;
            gpw(st)[2 * Rfull + row0 + b0 * 64 + lane] = V0;
        }
    } else {
        #ifndef ALVRL_EXP_NOBAR
        for (uint32_t k = 0; k < nch; k++) __syncthreads();
        #endif
    }
    if (wprof) {
        const bool n4 = NB == 4;
        padd(pbase + wv, pc_busy);
        padd(pbase + kWaves + wv, (long long)clock64() - wall0);
        padd(pbase + 2 * kWaves + wv, pc_red);
        padd(n4 ? PF_V_ISSUE : PF_V_RED, pc_sp[0]);
        padd(n4 ? PF_V_DATA : PF_P_STAGE, pc_sp[1]);
        padd(n4 ? PF_V_OWN : PF_V_COEF, pc_sp[2]);
        padd(n4 ? PF_V_CW : PF_V_REC, pc_sp[3]);
    }
    __syncthreads();
    if (!FU && glast && active && wv == (g == 0 ? 0 : 5)) {
        // the pass's final variances from every row's state (variance_passes_t, FU == false)
        const double* st = J.st + (size_t)g * 3 * Rfull;
        const double Wt = V.Wcur, rW = 1.0 / Wt;
        double pu = 0.0, pi = 0.0;
        for (uint32_t r = lane; r < Rfull; r += 64) {
            pu = pu + J.locw[r] * (gp(st)[Rfull + r] * rW);
            pi = pi + J.locw[r] * (gp(st)[2 * Rfull + r] * Wt);
        }
        pu = tree_d(pu);
        pi = tree_d(pi);
        if (lane == 0) {
            V.res_u = (float)pu; V.res_i = (float)pi;
            if (!isfinite(V.res_u) || V.res_u < 0) C.err = 1;
            if (!isfinite(V.res_i) || V.res_i < 0) C.err = 1;
        }
    }
    __syncthreads();
}

// One part of a divided split (PartJob): pass g (0 forward, 1 reverse) of
// variance_split_v3 over the row blocks [gb0, gb0 + nb) of the job (nb <= 7),
// with the whole workgroup on that pass: wave 0 forms the coefficients (the
// running weight total in the pass's column order, as every group of the
// one-workgroup engine does) and stores the row blocks' per-column totals to
// T instead of adding them; waves 1..nb run one 64-row block's recurrence
// each.  Per row and column the same IEEE operations in the same order as
// variance_split_v3 (rec below is its full-chunk and guarded paths), so the
// block totals are bit-identical to the ones that engine adds.
// FU = false (kPartInit): no prefix terms; the rows' final states go to
// pj.st and wave 0 stores the total weight to pj.wsum (variance_split_v3<false>).
// With nb <= 3 (FU) the halving trees leave the row waves: a row wave stores
// its half chunks' terms to LDS, and reducer wave nb + 1 + b runs block b's
// tree (the same tree8_transposed on the same values) one chunk later, so the
// coefficient wave stores chunk k - 2's totals at chunk k.  A part runs one
// wave per SIMD, where the trees' latency was the row wave's (var parts of a
// 100k-column split: 10.6 ms, against 7.2 ms for the tree-less init parts).
constexpr uint32_t kPartMaxBlk = 7;
constexpr uint32_t kPartRedMax = 3;   // row blocks whose trees run on reducer waves
static_assert(2 * kPartMaxBlk * 16 * sizeof(double) + 2 * sizeof(CoefBlock) + 2 * kPartRedMax * 2 * 8 * 64 * sizeof(double) <=
                  kPoolBytes, "variance part: pool");
template <bool FU>
__device__ __noinline__ void variance_part(const PartJob& pj, CC& cm_in, Ctl& C, const double* Tout_c, uint32_t g,
                                           uint32_t gb0, uint32_t nb, unsigned char* pool)
{
    CC& cm = uni(cm_in);
    double* const Tout = const_cast<double*>(Tout_c);
    const uint32_t Rt_rows = pj.nrows, m = pj.m, nblk_t = pj.nblk;
    const int tid = threadIdx.x, wv = tid >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const bool coefw = wv == 0;
    const uint32_t b0 = (uint32_t)wv - 1u;                       // row waves 1..nb: local block b0
    const bool roww = wv >= 1 && b0 < nb;
    const bool red = FU && cm.part_red && nb <= kPartRedMax;     // trees on reducer waves nb+1..2nb
    const uint32_t rb = (uint32_t)wv - 1u - nb;                  // a reducer's block
    const bool redw = red && wv >= 1 + (int)nb && rb < nb;
    double* Q = reinterpret_cast<double*>(pool);                 // [k & 1][kPartMaxBlk][16]
    CoefBlock* ring = reinterpret_cast<CoefBlock*>(pool + 2 * kPartMaxBlk * 16 * sizeof(double));
    // the row waves' terms for the reducers: [k & 1][block][half][8][lane]
    auto* const TH = lp(reinterpret_cast<double*>(pool + 2 * kPartMaxBlk * 16 * sizeof(double) + 2 * sizeof(CoefBlock)));
    auto th_at = [&](uint32_t k, uint32_t blk, uint32_t hsel, uint32_t i) {
        return ((((k & 1u) * kPartRedMax + blk) * 2u + hsel) * 8u + i) * 64u + lane;
    };
    const auto cwp = gp(pj.cw);
    const uint32_t nch = (m + kCH - 1) / kCH;
    const uint32_t nblk = (m + kCB64 - 1) / kCB64;
    auto cn_of = [&](uint32_t k) { return min((uint32_t)kCH, m - k * kCH); };
    auto ncol_of = [&](uint32_t b) { return min((uint32_t)kCB64, m - b * kCB64); };
    auto kw_of_blk = [&](uint32_t b) -> unsigned long long {
        if (b >= nblk) return 0ull;
        const uint32_t i = b * kCB64 + min(lane, ncol_of(b) - 1);
        return cwp[g == 0 ? i : m - 1 - i];
    };
    double W = 0.0, cWo = 0.0, cWn = 0.0, cw_w = 1.0;
    uint32_t cw_v = 0;
    unsigned long long kwN = 0;
    auto take = [&](unsigned long long kw, uint32_t b) {
        cw_v = (uint32_t)kw;
        cw_w = lane < ncol_of(b) ? (double)__uint_as_float((uint32_t)(kw >> 32)) : 1.0;
        cWo = 0.0; cWn = 0.0;
        if (lane < ncol_of(b)) ring[b & 1].vrl[lane] = cw_v;
    };
    if (coefw) {
        take(kw_of_blk(0), 0);
        for (uint32_t j = 0; j < 8; j++) coef_chain8(W, cw_w, j, ncol_of(0), cWo, cWn);
        coef_block_finish(C, cw_w, cWo, cWn, cw_v, ncol_of(0), &ring[0]);
        kwN = kw_of_blk(1);
    }
    __syncthreads();
    // rows past the job's last take its data at weight 0 (variance_split_v3)
    const uint32_t grow = (gb0 + (roww ? b0 : 0u)) * 64u + lane;
    const uint32_t r0 = min(grow, Rt_rows - 1);
    const RowRef rr0 = roww ? (pj.contig ? RowRef{(size_t)(pj.off0 + r0), (size_t)pj.stride0}
                                         : RowRef{(size_t)gp(pj.roff)[r0], (size_t)gp(pj.rstride)[r0]})
                            : RowRef{0, 0};
    const double lw0 = roww && grow < Rt_rows ? gp(pj.locw)[r0] : 0.0;
    // wave 0: the block totals of chunk kk to T[g][h][gb0 + b][n]
    auto store_totals = [&](uint32_t kk) {
        const uint32_t cn = cn_of(kk);
        const double* Qk = Q + (size_t)(kk & 1) * kPartMaxBlk * 16;
        const uint32_t sl = lane & 15, c = sl >> 1, h = sl & 1;
        const uint32_t n = kk * kCH + c;
        if (lane < 16 && c < cn) {
            double* const t = Tout + ((size_t)(g * 2 + h) * nblk_t + gb0) * m + n;
            for (uint32_t b = 0; b < nb; b++) gpw(t)[(size_t)b * m] = Qk[b * 16 + sl];
        }
    };
    auto rec = [&](uint32_t k, const float2* cur, uint32_t blk, double lw, double& sum0, double& M0, double& V0) {
        const uint32_t c0 = k * kCH, cn = cn_of(k);
        const CoefBlock& q = ring[(k / 8) & 1];
        const uint32_t o = (k % 8) * kCH;
        double th[kCH];
        auto half_done = [&](uint32_t hsel) {
            if (!FU) return;
            if (red) {
#pragma unroll
                for (uint32_t i = 0; i < 8; i++) TH[th_at(k, blk, hsel, i)] = th[i];
                return;
            }
            const double z = tree8_transposed(th, lane);
            if ((lane & 7) == 0) {
                const uint32_t h = lane >> 5, c = 4 * hsel + 2 * ((lane >> 3) & 1) + ((lane >> 4) & 1);
                Q[((size_t)(k & 1) * kPartMaxBlk + blk) * 16 + 2 * c + h] = z;
            }
        };
        if (cn == (uint32_t)kCH && k > 0) {
            struct CCol { double w, Wo, a, bb, rw, Wn, rWn; };
            auto ldc = [&](int c) {
                return CCol{q.w[o + c], q.Wo[o + c], q.a[o + c], q.bb[o + c], q.rw[o + c], q.Wn[o + c], q.rWn[o + c]};
            };
            auto col = [&](const CCol& k2, float2 e, double* t) {
                const double x = (double)e.x;
                const double tmp = k2.w * sum0 - k2.Wo * x;
                M0 = k2.a * M0 + k2.bb * (tmp * tmp);
                V0 = V0 + (double)e.y * k2.rw;
                sum0 = sum0 + x;
                if (FU) { t[0] = lw * (M0 * k2.rWn); t[1] = lw * (V0 * k2.Wn); }
            };
            CCol k0 = ldc(0), k1 = ldc(1), k2 = k1;
#pragma unroll
            for (int c = 0; c < kCH; c++) {
                if (c + 2 < kCH) k2 = ldc(c + 2);
                col(k0, cur[c], &th[2 * (c & 3)]);
                k0 = k1; k1 = k2;
                if (c == 3) half_done(0);
            }
            half_done(1);
        } else {
#pragma unroll
            for (int c = 0; c < kCH; c++) {
                double* t = &th[2 * (c & 3)];
                if ((uint32_t)c < cn) {
                    const double x = (double)cur[c].x;
                    const double tmp = q.w[o + c] * sum0 - q.Wo[o + c] * x;
                    if (c0 + c > 0) M0 = q.a[o + c] * M0 + q.bb[o + c] * (tmp * tmp);
                    V0 = V0 + (double)cur[c].y * q.rw[o + c];
                    sum0 = sum0 + x;
                    if (FU) { t[0] = lw * (M0 * q.rWn[o + c]); t[1] = lw * (V0 * q.Wn[o + c]); }
                } else if (FU) {
                    t[0] = 0.0; t[1] = 0.0;
                }
                if (c == 3) half_done(0);
                if (c == 7) half_done(1);
            }
        }
    };
    if (coefw) {
        // chunk k = 8B + j: store chunk k-1's block totals, form 8 columns of
        // block B+1's coefficients (the divisions at j = 7)
        for (uint32_t B = 0; B * 8 < nch; B++) {
            const uint32_t nbk = B + 1;
            if (nbk < nblk) take(kwN, nbk);
            kwN = kw_of_blk(nbk + 1);
#pragma unroll 1
            for (uint32_t j = 0; j < 8; j++) {
                const uint32_t k = B * 8 + j;
                if (k >= nch) break;
                if (FU && !red && k >= 1) store_totals(k - 1);
                if (red && k >= 2) store_totals(k - 2);
#ifndef ALVRL_EXPP_NOCOEF
                if (nbk < nblk) {
                    coef_chain8(W, cw_w, j, ncol_of(nbk), cWo, cWn);
                    if (j == 7 || k == nch - 1) coef_block_finish(C, cw_w, cWo, cWn, cw_v, ncol_of(nbk), &ring[nbk & 1]);
                }
#endif
#ifndef ALVRL_EXPP_NOBAR
                __syncthreads();
#endif
            }
        }
        if (red) {   // the reducers' last chunk
            if (nch >= 2) store_totals(nch - 2);
            __syncthreads();
        }
        if (FU) store_totals(nch - 1);
        else if (lane == 0 && gb0 == 0) gpw(pj.wsum)[0] = W;
    } else if (roww) {
        double sum0 = 0.0, M0 = 0.0, V0 = 0.0;
        float2 bufA[kCH], bufB[kCH], bufC[kCH];
        const float2* const Rt = cm.Rt + rr0.base;
        const size_t rstride = rr0.stride;
        auto load_chunk = [&](uint32_t k, float2* dst) {
            const uint32_t* ids = &ring[(k / 8) & 1].vrl[(k % 8) * kCH];
            const uint32_t cn = cn_of(k);
#ifdef ALVRL_EXPP_NOLOAD
#pragma unroll
            for (int c = 0; c < kCH; c++) dst[c] = make_float2((float)ids[(uint32_t)c < cn ? c : 0] * 1e-7f + (float)lane * 1e-9f, 0.25f);
#elif defined(ALVRL_EXPP_NOBAR)
#pragma unroll
            for (int c = 0; c < kCH; c++) dst[c] = ldg2(Rt, (size_t)min(ids[(uint32_t)c < cn ? c : 0], cm.nvrl - 1) * rstride);
#else
#pragma unroll
            for (int c = 0; c < kCH; c++) dst[c] = ldg2(Rt, (size_t)ids[(uint32_t)c < cn ? c : 0] * rstride);
#endif
        };
        load_chunk(0, bufA);
        load_chunk(min(1u, nch - 1), bufB);
        auto step = [&](uint32_t k, float2* cur, float2* pre) {
            load_chunk(min(k + 2, nch - 1), pre);
            rec(k, cur, b0, lw0, sum0, M0, V0);
#ifndef ALVRL_EXPP_NOBAR
            __syncthreads();
#endif
        };
        for (uint32_t k = 0; k < nch; k += 3) {
            step(k, bufA, bufC);
            if (k + 1 < nch) step(k + 1, bufB, bufA);
            if (k + 2 < nch) step(k + 2, bufC, bufB);
        }
        if (red) __syncthreads();
        if (!FU && grow < Rt_rows) {   // the row's final state (variance_split_v3<false>)
            gpw(pj.st)[Rt_rows + grow] = M0;
            gpw(pj.st)[2 * Rt_rows + grow] = V0;
        }
    } else if (redw) {
        // chunk k - 1's trees for block rb (half_done's tree and Q slots)
        auto reduce = [&](uint32_t k) {
#pragma unroll
            for (uint32_t hsel = 0; hsel < 2; hsel++) {
                double th[kCH];
#pragma unroll
                for (uint32_t i = 0; i < 8; i++) th[i] = TH[th_at(k, rb, hsel, i)];
                const double z = tree8_transposed(th, lane);
                if ((lane & 7) == 0) {
                    const uint32_t h = lane >> 5, c = 4 * hsel + 2 * ((lane >> 3) & 1) + ((lane >> 4) & 1);
                    Q[((size_t)(k & 1) * kPartMaxBlk + rb) * 16 + 2 * c + h] = z;
                }
            }
        };
        for (uint32_t k = 0; k < nch; k++) {
            if (k >= 1) reduce(k - 1);
#ifndef ALVRL_EXPP_NOBAR
            __syncthreads();
#endif
        }
        reduce(nch - 1);
        __syncthreads();
    } else {
#ifndef ALVRL_EXPP_NOBAR
        for (uint32_t k = 0; k < nch + (red ? 1u : 0u); k++) __syncthreads();
#endif
    }
    __syncthreads();
}

// The two passes of a small split (m <= kSmallMax columns, R <= 256 rows) in
// one step, without the chunk pipeline of variance_split_v3: waves 0-3 run
// the forward pass over row blocks 0-3, waves 4-7 the reverse one.  Wave 0
// (4) forms its pass's coefficients for all m columns (the running weight
// total in column order, one lane per column), every row wave then runs the
// recurrence over all m columns (its entries 8 columns ahead) and reduces
// each column's two prefix terms over its 64 rows with the halving tree
// (tree16_transposed); the block totals are added in ascending block order
// (wsum_blk).  The same IEEE operations in the same order as the oracle's
// cluster_variance and variance_split_v3, so the prefixes are bit-identical.
// Outputs stay in LDS: out[0..3][c] = fsu, fsi, feu, fei (prefix c of the
// forward / reverse pass; the forward u of prefix 0 is 0).
constexpr uint32_t kSmallMax = 256;
constexpr uint32_t kSmallBlocks = 14;                 // row blocks: up to 896 rows (row waves take blk, blk + 4, ...)
constexpr uint32_t kSmallCoefBytes = 2u * 7u * kSmallMax * 8u;
constexpr uint32_t kSmallVrlBytes = 2u * kSmallMax * 4u;
constexpr uint32_t kSmallQBytes = 2u * kSmallMax * 2u * kSmallBlocks * 8u;
constexpr uint32_t kSmallOutOff = kSmallCoefBytes + kSmallVrlBytes + kSmallQBytes;
static_assert(kSmallOutOff + 4u * kSmallMax * 4u <= kPoolBytes, "small split engine exceeds the LDS pool");
__device__ __forceinline__ const float* small_out(const unsigned char* pool) { return reinterpret_cast<const float*>(pool + kSmallOutOff); }
__device__ __noinline__ void variance_split_small(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* base,
                                                  uint32_t m, unsigned char* pool)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    m = (uint32_t)__builtin_amdgcn_readfirstlane((int)m);   // uniform: scalar loop and guard branches
    const uint32_t R = J.nrows, NB = (R + 63) / 64;
    const int tid = threadIdx.x, wv = tid >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const int g = wv >> 2;                              // 0: forward, 1: reverse
    if (!LDS_OK(m <= kSmallMax && NB <= kSmallBlocks, "small split size", m, NB)) return;
    const uint32_t blk = (uint32_t)(wv & 3);
    auto* const coef = lp(reinterpret_cast<double*>(pool));                          // [g][7][kSmallMax]
    auto* const vr = lp(reinterpret_cast<uint32_t*>(pool + kSmallCoefBytes));        // [g][kSmallMax]
    auto* const Q = lp(reinterpret_cast<double*>(pool + kSmallCoefBytes + kSmallVrlBytes));   // [g][c][h][blk]
    auto* const out = lp(reinterpret_cast<float*>(pool + kSmallOutOff));             // [g * 2 + h][c]
    auto* const cg = coef + (size_t)g * 7 * kSmallMax;
    auto* const vg = vr + (size_t)g * kSmallMax;
    if (blk == 0) {
        // chunk_coefs (:1075-1085): W before / after each column's weight
        double W = 0.0;
        for (uint32_t c0 = 0; c0 < m; c0 += 64) {
            const uint32_t c = c0 + lane;
            const bool has = c < m;
            const uint32_t i = has ? c : m - 1;
            const uint32_t v = gp(base)[g == 0 ? i : m - 1 - i];
            const double w = (double)gp(J.colw)[v];
            const uint32_t n = min(64u, m - c0);
            double Wo = 0.0, Wn = 0.0;
            for (uint32_t k = 0; k < n; k++) {
                const double wk = readlane_d(w, k);
                const bool me = lane == k;
                Wo = me ? W : Wo;
                W = W + wk;
                Wn = me ? W : Wn;
            }
            if (has) {
                if (!isfinite(w) || w <= 0) C.err = 1;
                const double rw = 1.0 / w;
                cg[c] = w;
                cg[kSmallMax + c] = Wo;
                cg[2 * kSmallMax + c] = (Wn * Wn) / (Wo * Wo);
                cg[3 * kSmallMax + c] = (rw + 1.0 / Wo);
                cg[4 * kSmallMax + c] = rw;
                cg[5 * kSmallMax + c] = Wn;
                cg[6 * kSmallMax + c] = 1.0 / Wn;
                vg[c] = v;
            }
        }
    }
    __syncthreads();
    // row wave blk runs row blocks blk, blk + 4, ... (more than 256 rows: one
    // after the other, each from a zero state)
    for (uint32_t bb = blk; bb < NB; bb += 4) {
        const bool valid = bb * 64 + lane < R;
        const uint32_t r = min(bb * 64 + lane, R - 1);
        const RowRef rr = row_ref(J, r);
        const double lw = J.locw[r];
        const float2* const Rt = cm.Rt + rr.base;
        const size_t rs = rr.stride;
        double sum = 0.0, M = 0.0, V = 0.0;
        float2 bufA[kCH], bufB[kCH];
        auto load = [&](uint32_t c0, float2* d) {
#pragma unroll
            for (int q = 0; q < kCH; q++) d[q] = ldg2(Rt, (size_t)vg[min(c0 + (uint32_t)q, m - 1)] * rs);
        };
        auto chunk = [&](uint32_t c0, const float2* cur) {
            double tv[2 * kCH];
#pragma unroll
            for (int q = 0; q < kCH; q++) {
                const uint32_t c = c0 + (uint32_t)q;
                if (c < m) {
                    const double x = (double)cur[q].x;
                    const double tmp = cg[c] * sum - cg[kSmallMax + c] * x;
                    if (c > 0) M = cg[2 * kSmallMax + c] * M + cg[3 * kSmallMax + c] * (tmp * tmp);
                    V = V + (double)cur[q].y * cg[4 * kSmallMax + c];
                    sum = sum + x;
                    tv[2 * q] = lw * (M * cg[6 * kSmallMax + c]);
                    tv[2 * q + 1] = lw * (V * cg[5 * kSmallMax + c]);
                } else {
                    tv[2 * q] = 0.0; tv[2 * q + 1] = 0.0;
                }
            }
#pragma unroll
            for (int i = 0; i < 2 * kCH; i++) tv[i] = valid ? tv[i] : 0.0;
            const double z = tree16_transposed(tv, lane);
            if ((lane & 3) == 0) {
                const uint32_t h = lane >> 5, c = 4 * ((lane >> 2) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 4) & 1);
                if (c0 + c < m) Q[(((size_t)g * kSmallMax + c0 + c) * 2 + h) * kSmallBlocks + bb] = z;
            }
        };
        // three chunks' entries issued together (clamped: past the end the
        // last chunk again), then the three chunks.  Loads issued under a
        // branch, or in flight across the loop's back edge, make the compiler
        // wait for every load in flight (it cannot match them across paths)
        const uint32_t nch = (m + kCH - 1) / kCH;
        float2 bufC[kCH];
        for (uint32_t k = 0; k < nch; k += 3) {
            load(k * kCH, bufA);
            load(min(k + 1, nch - 1) * kCH, bufB);
            load(min(k + 2, nch - 1) * kCH, bufC);
            chunk(k * kCH, bufA);
            if (k + 1 < nch) chunk((k + 1) * kCH, bufB);
            if (k + 2 < nch) chunk((k + 2) * kCH, bufC);
        }
    }
    __syncthreads();
    // block totals in ascending block order (wsum_blk), as floats
    VarGroup* const vgrp = C.vg;
    for (uint32_t t = (uint32_t)tid; t < 4 * m; t += kThreads) {
        const uint32_t gh = t / m, c = t - gh * m, gg = gh >> 1, h = gh & 1;
        const auto* q = Q + (((size_t)gg * kSmallMax + c) * 2 + h) * kSmallBlocks;
        double acc = q[0];
        for (uint32_t b = 1; b < NB; b++) acc = acc + q[b];
        const float f = (h == 0 && c == 0) ? 0.0f : (float)acc;
        out[gh * kSmallMax + c] = f;
        if (c == m - 1) {
            if (h == 0) vgrp[gg].res_u = f; else vgrp[gg].res_i = f;
            if (!isfinite(f) || f < 0) C.err = 1;
        }
    }
    __syncthreads();
}

__device__ __noinline__ bool split_parts(CJ& J, CC& cm, Ctl& C, const uint32_t* base, uint32_t m,
                            float* fu0, float* fi0, float* fu1, float* fi1, unsigned char* pool);
__device__ bool proj_parts(CJ& J, CC& cm, Ctl& C, uint32_t begin, uint32_t m, unsigned char* pool);
__device__ bool init_parts(CJ& J, CC& cm, Ctl& C, const uint32_t* base, uint32_t m, unsigned char* pool);
__device__ bool colw_parts(CJ& J, CC& cm, Ctl& C, uint32_t vb, uint32_t ve, unsigned char* pool);
__device__ void variance_passes(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* base, uint32_t m,
                                int npass, float* fu0, float* fi0, float* fu1, float* fi1, unsigned char* pool,
                                Prof* pf = nullptr)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    // a large split in parts on idle workgroups (split_parts), when a slot is free
    const uint32_t pmin = J.nrows > 256 ? cm.part_min_tall : cm.part_min;   // 0: never
    if (fu0 && npass == 2 && cm.parts && cm.var_v3 && pmin && m >= pmin &&
        split_parts(J, cm, C, base, m, fu0, fi0, fu1, fi1, pool))
        return;
    if (!fu0 && npass == 1 && cm.parts && cm.var_v3 && pmin && m >= pmin &&
        init_parts(J, cm, C, base, m, pool))
        return;
    const uint32_t NB = (J.nrows + 63) / 64;
    if (pf && (!pf->p || threadIdx.x != 0)) pf = nullptr;
    const bool lds = (size_t)2 * 2 * kCH * NB * 64 * sizeof(double2) <= kPoolBytes;
    if (NB > 4 && cm.var_v3 && J.carry && (fu0 ? npass == 2 : true)) {
        // more than 256 rows: the v3 engine once per group of <= 256 rows, the
        // block-ordered row sums carried from group to group (wsum_blk's order
        // over all the blocks), the prefix results written by the last group
        const uint32_t G = (J.nrows + 255) / 256;
        for (uint32_t gr = 0; gr < G; gr++) {
            if (threadIdx.x == 0) {
                C.g_row0 = gr * 256u; C.g_first = gr == 0; C.g_last = gr + 1 == G; C.g_carry = J.carry;
            }
            __syncthreads();
            if (fu0) variance_split_v3<true, true>(J, cm, C, base, m, 2, fu0, fi0, fu1, fi1, pool);
            else variance_split_v3<false, true>(J, cm, C, base, m, npass, nullptr, nullptr, nullptr, nullptr, pool);
        }
        if (threadIdx.x == 0) { C.g_row0 = 0; C.g_first = 1; C.g_last = 1; C.g_carry = nullptr; }
        __syncthreads();
        return;
    }
    if (fu0 && npass == 2 && NB <= 4 && cm.var_v3) {
        variance_split_v3<true>(J, cm, C, base, m, 2, fu0, fi0, fu1, fi1, pool);
        return;
    }
    if (!fu0 && NB <= 4 && cm.var_v3) {
        variance_split_v3<false>(J, cm, C, base, m, npass, nullptr, nullptr, nullptr, nullptr, pool);
        return;
    }
    if (fu0) {
        if (lds) variance_passes_t<true, true>(J, cm, C, base, m, npass, fu0, fi0, fu1, fi1, pool, pf);
        else variance_passes_t<false, true>(J, cm, C, base, m, npass, fu0, fi0, fu1, fi1, pool, pf);
    } else {
        if (lds) variance_passes_t<true, false>(J, cm, C, base, m, npass, fu0, fi0, fu1, fi1, pool, pf);
        else variance_passes_t<false, false>(J, cm, C, base, m, npass, fu0, fi0, fu1, fi1, pool, pf);
    }
}

__device__ __forceinline__ unsigned char* pool_end(void* pool) { return reinterpret_cast<unsigned char*>(pool) + kPoolBytes; }

// Column reductions over the rows, one wave per column, kCB columns per wave
// at a time (their loads in flight together), rows in the shared order.
constexpr int kCB = 8;
constexpr int kRB = 4;                 // row blocks kept in registers (R <= 256)

// ------------------------------------------------------------- sort --
__device__ __forceinline__ unsigned long long proj_key(float p, uint32_t vrl)
{
    if (p == 0.0f) p = 0.0f;   // -0 == +0 for std::pair's operator<
    uint32_t u = __float_as_uint(p);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ((unsigned long long)u << 32) | vrl;
}

// Sorts J.keys0[0..m); returns the buffer holding the result.
typedef __attribute__((address_space(1))) unsigned long long glb_u64;

// Bitonic sort of n <= kBitonicMax keys in LDS: in[0..n) -> out[0..n)
__device__ __forceinline__ void bitonic_lds(lds_u64* lds, const glb_u64* in, glb_u64* out, uint32_t n)
{
    const int tid = threadIdx.x;
    uint32_t n2 = 1;
    while (n2 < n) n2 <<= 1;
    if (!LDS_OK(n2 <= (uint32_t)kBitonicMax, "bitonic keys", n2, kBitonicMax)) return;
    for (uint32_t i = tid; i < n2; i += kThreads) lds[i] = i < n ? in[i] : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = tid; i < n2; i += kThreads) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long a = lds[i], b = lds[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) { lds[i] = b; lds[ixj] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = tid; i < n; i += kThreads) out[i] = lds[i];
    __syncthreads();
}

// 1-bit LSD radix over the bits that vary, n keys in src (dst: scratch of
// the same size); returns the array that holds the sorted keys
__device__ glb_u64* radix_sort(Ctl& C, glb_u64* src, glb_u64* dst, uint32_t n)
{
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    auto* const Cn = lp(&C.cnt[0]);
    if (tid == 0) { C.lo_or = 0; C.hi_or = 0; C.lo_and = 0xFFFFFFFFu; C.hi_and = 0xFFFFFFFFu; }
    __syncthreads();
    {
        uint32_t lo_o = 0, hi_o = 0, lo_a = 0xFFFFFFFFu, hi_a = 0xFFFFFFFFu;
        for (uint32_t i = tid; i < n; i += kThreads) {
            const unsigned long long k = src[i];
            lo_o |= (uint32_t)k; hi_o |= (uint32_t)(k >> 32);
            lo_a &= (uint32_t)k; hi_a &= (uint32_t)(k >> 32);
        }
        atomicOr(&C.lo_or, lo_o); atomicOr(&C.hi_or, hi_o);
        atomicAnd(&C.lo_and, lo_a); atomicAnd(&C.hi_and, hi_a);
    }
    __syncthreads();
    const unsigned long long vary = (((unsigned long long)(C.hi_or ^ C.hi_and)) << 32) |
                                    (unsigned long long)(C.lo_or ^ C.lo_and);
    for (int bit = 0; bit < 64; bit++) {
        if (!((vary >> bit) & 1ull)) continue;
        if (tid == 0) C.zeros = 0;
        __syncthreads();
        uint32_t z = 0;
        for (uint32_t i = tid; i < n; i += kThreads) z += ((src[i] >> bit) & 1ull) ? 0u : 1u;
        atomicAdd(&C.zeros, z);
        __syncthreads();
        const uint32_t zeros = C.zeros;
        uint32_t zbase = 0, obase = zeros;
        for (uint32_t t0 = 0; t0 < n; t0 += kThreads) {
            const uint32_t i = t0 + tid;
            const bool valid = i < n;
            const unsigned long long k = valid ? src[i] : 0ull;
            const bool one = valid && ((k >> bit) & 1ull);
            const bool zero = valid && !one;
            const unsigned long long bz = __ballot(zero), bo = __ballot(one);
            const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            const uint32_t rz = __popcll(bz & lt), ro = __popcll(bo & lt);
            if (lane == 0) Cn[wave] = (uint32_t)__popcll(bz) | ((uint32_t)__popcll(bo) << 16);
            __syncthreads();
            uint32_t pz = 0, po = 0, tz = 0, to = 0;
            for (int w = 0; w < kWaves; w++) {
                const uint32_t cz = Cn[w] & 0xFFFFu, co = Cn[w] >> 16;
                if (w < wave) { pz += cz; po += co; }
                tz += cz; to += co;
            }
            if (zero) dst[zbase + pz + rz] = k;
            if (one) dst[obase + po + ro] = k;
            zbase += tz; obase += to;
            __syncthreads();
        }
        auto* t = src; src = dst; dst = t;
    }
    return src;
}

// LSD radix sort of n unique keys, digits of <= 8 bits over the bit ranges
// that vary (the low and the high word separately: a projection key's
// vrl id and its orderable float each span a run of bits).  Each wave owns a
// contiguous 1/8 of the array and keeps its own count per digit, so a pass
// has no barrier inside it: a key's place is its digit's offset for the
// wave (the scan of counts in (digit, wave) order) plus its rank among the
// batch's lanes with the same digit (ballots per digit bit), which keeps the
// sort stable.  The scatter also counts the next pass's digits per owner of
// the destination.  Every loop keeps 8 (the scatter 16) loads per lane in
// flight.  LDS: counts[2][256][8], offsets[256][8] (24 KB of
// the pool).  Keys in a; b is scratch of n keys; returns the array holding
// the sorted keys.
__device__ __noinline__ glb_u64* radix8_sort(Ctl& C_in, glb_u64* a, glb_u64* b, uint32_t n, unsigned char* pool)
{
    const int tid = threadIdx.x;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = (uint32_t)(tid & 63);
    auto& C = *lp(&C_in);
    auto* const cnt = lp(reinterpret_cast<uint32_t*>(pool));   // [2][256 * 8]
    auto* const off = cnt + 2 * 2048;                           // [256 * 8]
    auto* const wsum = off + 2048;                              // [8]
    n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n);
    constexpr uint32_t B = 8;
    // the bits that vary
    if (tid == 0) { C.lo_or = 0; C.hi_or = 0; C.lo_and = 0xFFFFFFFFu; C.hi_and = 0xFFFFFFFFu; }
    __syncthreads();
    {
        uint32_t lo_o = 0, hi_o = 0, lo_a = 0xFFFFFFFFu, hi_a = 0xFFFFFFFFu;
        for (uint32_t i0 = 0; i0 < n; i0 += B * kThreads) {
            unsigned long long k[B];
#pragma unroll
            for (uint32_t j = 0; j < B; j++) k[j] = a[min(i0 + j * kThreads + (uint32_t)tid, n - 1)];   // a repeat is harmless
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                lo_o |= (uint32_t)k[j]; hi_o |= (uint32_t)(k[j] >> 32);
                lo_a &= (uint32_t)k[j]; hi_a &= (uint32_t)(k[j] >> 32);
            }
        }
        __hip_atomic_fetch_or(&C.lo_or, lo_o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_or(&C.hi_or, hi_o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_and(&C.lo_and, lo_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_and(&C.hi_and, hi_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    for (uint32_t i = (uint32_t)tid; i < 2048; i += kThreads) cnt[i] = 0;
    __syncthreads();
    const uint32_t vlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(C.lo_or ^ C.lo_and));
    const uint32_t vhi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(C.hi_or ^ C.hi_and));
    // digit windows: nl over the low word's varying run, nh over the high word's
    const uint32_t l0 = vlo ? (uint32_t)__builtin_ctz(vlo) : 0u, l1 = vlo ? 32u - (uint32_t)__builtin_clz(vlo) : 0u;
    const uint32_t h0 = vhi ? (uint32_t)__builtin_ctz(vhi) : 0u, h1 = vhi ? 32u - (uint32_t)__builtin_clz(vhi) : 0u;
    const uint32_t nl = (l1 - l0 + 7) / 8, nh = (h1 - h0 + 7) / 8;
    const uint32_t wl = nl ? (l1 - l0 + nl - 1) / nl : 0u, wh = nh ? (h1 - h0 + nh - 1) / nh : 0u;
    const uint32_t P = nl + nh;
    auto win = [&](uint32_t p, uint32_t& sh, uint32_t& w) {
        if (p < nl) { sh = l0 + p * wl; w = min(wl, l1 - sh); }
        else { sh = 32u + h0 + (p - nl) * wh; w = min(wh, 32u + h1 - sh); }
    };
    // each wave's segment: S keys (a multiple of 64), the last ones shorter
    const uint32_t S = ((n + 8u * 64u - 1) / (8u * 64u)) * 64u;
    const float rS = 1.0f / (float)S;
    auto seg_of = [&](uint32_t o) {   // o / S without a division
        uint32_t g = min(7u, (uint32_t)((float)o * rS));
        g = g * S > o ? g - 1u : g;
        g = g < 7u && (g + 1u) * S <= o ? g + 1u : g;
        return g;
    };
    const uint32_t sb = min(n, wave * S), se = min(n, sb + S);
    if (P > 0 && sb < se) {   // the first pass's counts
        uint32_t sh, w;
        win(0, sh, w);
        const uint32_t mask = (1u << w) - 1u;
        for (uint32_t i0 = sb; i0 < se; i0 += B * 64) {
            unsigned long long k[B];
#pragma unroll
            for (uint32_t j = 0; j < B; j++) k[j] = a[min(i0 + j * 64 + lane, se - 1)];
#pragma unroll
            for (uint32_t j = 0; j < B; j++)
                if (i0 + j * 64 + lane < se)
                    __hip_atomic_fetch_add(&cnt[((uint32_t)(k[j] >> sh) & mask) * 8 + wave], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    glb_u64* src = a;
    glb_u64* dst = b;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t p = 0; p < P; p++) {
        uint32_t sh, w, sh2 = 0, w2 = 1;
        win(p, sh, w);
        const bool more = p + 1 < P;
        if (more) win(p + 1, sh2, w2);
        const uint32_t mask = (1u << w) - 1u, mask2 = (1u << w2) - 1u;
        auto* const cc = cnt + (p & 1) * 2048;
        auto* const cn = cnt + ((p + 1) & 1) * 2048;
        // exclusive scan of the counts in (digit, wave) order: 4 per thread
        {
            const uint32_t i0 = (uint32_t)tid * 4;
            const uint32_t c0 = cc[i0], c1 = cc[i0 + 1], c2 = cc[i0 + 2], c3 = cc[i0 + 3];
            const uint32_t t = c0 + c1 + c2 + c3;
            uint32_t x = t;   // inclusive scan over the wave
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
                if (lane >= (uint32_t)d) x += y;
            }
            if (lane == 63) wsum[wave] = x;
            __syncthreads();
            uint32_t base = 0;
            for (uint32_t v = 0; v < wave; v++) base += wsum[v];
            const uint32_t e0 = base + x - t;
            off[i0] = e0; off[i0 + 1] = e0 + c0; off[i0 + 2] = e0 + c0 + c1; off[i0 + 3] = e0 + c0 + c1 + c2;
            cn[i0] = 0; cn[i0 + 1] = 0; cn[i0 + 2] = 0; cn[i0 + 3] = 0;   // the next pass's counts
        }
        __syncthreads();
        // the scatter: 8 batches of 64 keys per step, the next step's loaded
        // before this one's are placed
        auto ld = [&](uint32_t base, unsigned long long* k) {
#pragma unroll
            for (uint32_t j = 0; j < B; j++) k[j] = src[min(base + j * 64 + lane, se - 1)];
        };
        auto place = [&](uint32_t base, const unsigned long long* k) {
#pragma unroll
            for (uint32_t j = 0; j < B; j++) {
                const uint32_t i = base + j * 64;
                if (i >= se) break;
                const bool valid = i + lane < se;
                const uint32_t d = (uint32_t)(k[j] >> sh) & mask;
                unsigned long long mm = __ballot(valid);
#pragma unroll
                for (uint32_t bt = 0; bt < 8; bt++) {
                    if (bt < w) {
                        const bool one = (d >> bt) & 1u;
                        const unsigned long long bl = __ballot(one);
                        mm &= one ? bl : ~bl;
                    }
                }
                const uint32_t rank = (uint32_t)__popcll(mm & lt);
                const uint32_t ob = off[d * 8 + wave];
                const uint32_t o = ob + rank;
                if (valid) {
                    dst[o] = k[j];
                    if ((mm >> lane) == 1ull) off[d * 8 + wave] = ob + (uint32_t)__popcll(mm);
                    if (more) {
                        const uint32_t d2 = (uint32_t)(k[j] >> sh2) & mask2;
                        __hip_atomic_fetch_add(&cn[d2 * 8 + seg_of(o)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        };
        // (two sets loaded at the top of each step and placed within it: a
        // load in flight across the loop's back edge costs a full drain)
        constexpr uint32_t ST = B * 64;
        for (uint32_t base = sb; base < se; base += 2 * ST) {
            unsigned long long kA[B], kB[B];
            ld(base, kA);
            ld(base + ST, kB);
            place(base, kA);
            place(base + ST, kB);
        }
        __syncthreads();
        glb_u64* const t = src; src = dst; dst = t;
    }
    return src;
}

// The projection sort of split() (:641-648): sorts keys0[0..m) in place
// (keys are unique, so every correct sort gives the same order).  Up to
// kBitonicMax keys: one bitonic sort in LDS.  Larger clusters: a bucket pass
// on the projection value (monotone: bucket = floor((p - pmin) * NB /
// (pmax - pmin)), non-finite values at the ends) scatters the keys into
// buckets of ~4k, each then sorted in LDS (a bucket above kBitonicMax, e.g.
// many equal projections, takes the radix sort).
constexpr uint32_t kSortBuckets = 1024;
constexpr uint32_t kSortCtlBytes = 2 * kSortBuckets * 4;                 // counts, cursors
constexpr uint32_t kBucketSortMax = (kPoolBytes - kSortCtlBytes) / 8 >= (uint32_t)kBitonicMax ? (uint32_t)kBitonicMax : 8192u;
__device__ __forceinline__ float key_proj(uint32_t u)
{
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
__device__ ALVRL_PROJ_INL unsigned long long* sort_keys(CJ& J_in, Ctl& C, uint32_t m, unsigned long long* lds_g,
                                                     uint32_t radix_min)
{
    CJ& J = uni(J_in);
    const int tid = threadIdx.x;
    auto* const k0 = gpw(J.keys0);
    auto* const k1 = gpw(J.keys1);
    if (m >= radix_min) {   // the result in keys0: a later phase writes keys1
        const glb_u64* r = radix8_sort(C, k0, k1, m, reinterpret_cast<unsigned char*>(lds_g));
        if (r != k0) {
            for (uint32_t i = tid; i < m; i += kThreads) k0[i] = r[i];
            __syncthreads();
        }
        return J.keys0;
    }
    if (m <= (uint32_t)kBitonicMax) {
        bitonic_lds(lp(lds_g), k0, k0, m);
        return J.keys0;
    }
    auto* const cnt = lp(reinterpret_cast<uint32_t*>(lds_g));
    auto* const cur = cnt + kSortBuckets;
    auto lds_inc = [](__attribute__((address_space(3))) uint32_t* p) {
        return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    lds_u64* const lds = lp(lds_g) + kSortCtlBytes / 8;
    const uint32_t NB = min(kSortBuckets, (m + 4095) / 4096);
    // finite range of the projections, as key words (monotone in p)
    if (tid == 0) { C.lo_and = 0xFFFFFFFFu; C.hi_or = 0; }
    for (uint32_t b = tid; b < NB; b += kThreads) cnt[b] = 0;
    __syncthreads();
    {
        uint32_t lo = 0xFFFFFFFFu, hi = 0;
        for (uint32_t i = tid; i < m; i += kThreads) {
            const uint32_t u = (uint32_t)(k0[i] >> 32);
            if (isfinite(key_proj(u))) { lo = min(lo, u); hi = max(hi, u); }
        }
        atomicMin(&C.lo_and, lo); atomicMax(&C.hi_or, hi);
    }
    __syncthreads();
    const uint32_t ulo = C.lo_and, uhi = C.hi_or;
    const bool any = ulo <= uhi;
    const float plo = any ? key_proj(ulo) : 0.0f, phi = any ? key_proj(uhi) : 0.0f;
    const float scale = phi > plo ? (float)NB / (phi - plo) : 0.0f;
    auto bucket = [&](uint32_t u) -> uint32_t {
        if (!any || u < ulo) return 0u;
        if (u > uhi) return NB - 1;
        const float x = (key_proj(u) - plo) * scale;
        return min(NB - 1, (uint32_t)max(0.0f, x));
    };
    for (uint32_t i = tid; i < m; i += kThreads) lds_inc(&cnt[bucket((uint32_t)(k0[i] >> 32))]);
    __syncthreads();
    if (tid == 0) {
        uint32_t o = 0;
        for (uint32_t b = 0; b < NB; b++) { cur[b] = o; o += cnt[b]; }
    }
    __syncthreads();
    for (uint32_t i = tid; i < m; i += kThreads) {
        const unsigned long long k = k0[i];
        k1[lds_inc(&cur[bucket((uint32_t)(k >> 32))])] = k;
    }
    __syncthreads();
    // cur[b] is now the end of bucket b
    for (uint32_t b = 0; b < NB; b++) {
        const uint32_t e = cur[b], n = cnt[b], o = e - n;
        if (n == 0) continue;
        if (n <= kBucketSortMax) {
            bitonic_lds(lds, k1 + o, k0 + o, n);
        } else {
            glb_u64* r = radix_sort(C, k1 + o, k0 + o, n);
            if (r != k0 + o) {
                for (uint32_t i = tid; i < n; i += kThreads) k0[o + i] = r[i];
                __syncthreads();
            }
        }
    }
    return J.keys0;
}

// The projections of a range of a divided split's columns (proj_parts):
// split_projections' arithmetic over columns [jb, je) of pj.ids[0..m), each
// column's key depends on that column alone.  (split() keeps its own
// JobDev-based split_projections below: routing every split through this
// function cost 10 ms of the C4 refinement -- 309 against 300 ms, same box,
// profiles/r04/parts/r4u_summary.txt -- from the code it changed around the
// calls, not from the projections themselves.)
__device__ __forceinline__ RowRef row_ref(const PartJob& pj, uint32_t r)
{
    return pj.contig ? RowRef{(size_t)(pj.off0 + r), (size_t)pj.stride0}
                     : RowRef{(size_t)gp(pj.roff)[r], (size_t)gp(pj.rstride)[r]};
}
__device__ __noinline__ void proj_range(const PartJob& pj, CC& cm_in, uint32_t jb, uint32_t je)
{
    CC& cm = uni(cm_in);
    jb = (uint32_t)__builtin_amdgcn_readfirstlane((int)jb);   // uniform: scalar loop exits
    je = (uint32_t)__builtin_amdgcn_readfirstlane((int)je);
    const uint32_t R = pj.nrows;
    const int wave = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = kWaves * kCB;
    const float2* const Rt = cm.Rt;                  // register copy (cm is behind a generic pointer)
    auto* const k0 = gpw(pj.keys);
    const auto* const vrls = gp(pj.ids);
    const auto* const dir = gp(pj.dir);
    if (R <= 64u * kRB) {
        float d[kRB];
        RowRef row[kRB];
#pragma unroll
        for (int rb = 0; rb < kRB; rb++) {
            const uint32_t r = lane + 64u * rb;
            d[rb] = r < R ? dir[r] : 0.0f;
            row[rb] = row_ref(pj, r < R ? r : 0);
        }
        // ids two steps ahead, entries one step ahead, every load issued (see
        // split_projections)
        auto ldid = [&](uint32_t j0, uint32_t* v) {
#pragma unroll
            for (int q = 0; q < kCB; q++) v[q] = vrls[min(j0 + (uint32_t)q, je - 1)];
        };
        auto ldx = [&](const uint32_t* v, float (*x)[kCB]) {
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
#pragma unroll
                for (int q = 0; q < kCB; q++) x[rb][q] = ldg2(Rt, row[rb].base + (size_t)v[q] * row[rb].stride).x;
        };
        auto reduce = [&](uint32_t j0, const uint32_t* v, float (*x)[kCB]) {
            float pn[kCB], pp[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) { pn[q] = 0.0f; pp[q] = 0.0f; }
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
                if (lane + 64u * rb < R) {
#pragma unroll
                    for (int q = 0; q < kCB; q++) { const float a = fabsf(x[rb][q]); pn[q] = pn[q] + a * a; }
                }
            tree_fn<kCB>(pn);
            float nc[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) nc[q] = sqrtf(__shfl(pn[q], 0, 64));
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
                if (lane + 64u * rb < R) {
#pragma unroll
                    for (int q = 0; q < kCB; q++) pp[q] = pp[q] + d[rb] * (x[rb][q] / nc[q]);
                }
            tree_fn<kCB>(pp);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < kCB; q++)
                    if (j0 + q < je) k0[j0 + q] = proj_key(nc[q] != 0 ? pp[q] : 0.0f, v[q]);
            }
        };
        uint32_t j0 = jb + (uint32_t)wave * kCB;
        if (j0 < je) {
            const uint32_t jl = j0 + ((je - 1 - j0) / stride) * stride;   // the wave's last batch
            auto cl = [&](uint32_t j) { return min(j, jl); };
            uint32_t kA[kCB], kB[kCB], vN[kCB];
            float xA[kRB][kCB], xB[kRB][kCB];
            ldid(j0, vN);
#pragma unroll
            for (int q = 0; q < kCB; q++) kA[q] = vN[q];
            ldid(cl(j0 + stride), vN);
            ldx(kA, xA);
            for (;; j0 += 2 * stride) {
#pragma unroll
                for (int q = 0; q < kCB; q++) kB[q] = vN[q];
                ldid(cl(j0 + 2 * stride), vN);
                ldx(kB, xB);
                reduce(j0, kA, xA);
                if (j0 + stride >= je) break;
#pragma unroll
                for (int q = 0; q < kCB; q++) kA[q] = vN[q];
                ldid(cl(j0 + 3 * stride), vN);
                ldx(kA, xA);
                reduce(j0 + stride, kB, xB);
                if (j0 + 2 * stride >= je) break;
            }
        }
    } else {                                // tall local matrices: two passes from memory
        for (uint32_t j0 = jb + (uint32_t)wave * kCB; j0 < je; j0 += stride) {
            uint32_t vr[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) vr[q] = vrls[min(j0 + (uint32_t)q, je - 1)];
            float pn[kCB], pp[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) { pn[q] = 0.0f; pp[q] = 0.0f; }
            for (uint32_t r = lane; r < R; r += 64) {
                const RowRef rw = row_ref(pj, r);
#pragma unroll
                for (int q = 0; q < kCB; q++) { const float a = fabsf(ldg2(Rt, rw.base + (size_t)vr[q] * rw.stride).x); pn[q] = pn[q] + a * a; }
            }
            float nc[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) nc[q] = sqrtf(__shfl(tree_f(pn[q]), 0, 64));
            for (uint32_t r = lane; r < R; r += 64) {
                const RowRef rw = row_ref(pj, r);
                const float dd = dir[r];
#pragma unroll
                for (int q = 0; q < kCB; q++) pp[q] = pp[q] + dd * (ldg2(Rt, rw.base + (size_t)vr[q] * rw.stride).x / nc[q]);
            }
#pragma unroll
            for (int q = 0; q < kCB; q++) {
                const float pr = tree_f(pp[q]);
                if (lane == 0 && j0 + q < je) k0[j0 + q] = proj_key(nc[q] != 0 ? pr : 0.0f, vr[q]);
            }
        }
    }
}
__device__ __forceinline__ PartJob part_job(CJ& J)
{
    PartJob pj{};
    pj.roff = J.roff; pj.rstride = J.rstride; pj.off0 = J.off0; pj.stride0 = J.stride0; pj.contig = J.contig;
    pj.locw = J.locw; pj.nrows = J.nrows;
    return pj;
}
// Projections of split() (:625-640): one wave per column, kCB columns per
// batch, rows in the shared order (norm, then the normalised dot product with
// the split direction).  For R <= 64*kRB the batch's entries stay in
// registers for both sums and the next batch's loads are in flight while
// the current one is reduced (ping-pong buffers, no copies).
__device__ ALVRL_PROJ_INL void split_projections(CJ& J_in, CC& cm_in, uint32_t begin, uint32_t m)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    begin = (uint32_t)__builtin_amdgcn_readfirstlane((int)begin);   // uniform: scalar loop exits
    m = (uint32_t)__builtin_amdgcn_readfirstlane((int)m);
    const uint32_t R = J.nrows;
    const int wave = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = kWaves * kCB;
    const float2* const Rt = cm.Rt;                  // register copy (cm is behind a generic pointer)
    auto* const k0 = gpw(J.keys0);
    const auto* const vrls = gp(J.vrls);
    const auto* const dir = gp(J.dir);
    if (R <= 64u * kRB) {
        float d[kRB];
        RowRef row[kRB];
#pragma unroll
        for (int rb = 0; rb < kRB; rb++) {
            const uint32_t r = lane + 64u * rb;
            d[rb] = r < R ? dir[r] : 0.0f;
            row[rb] = row_ref(J, r < R ? r : 0);
        }
        // a batch's ids are loaded two steps ahead and its entries one step
        // ahead, every load issued (clamped to the wave's last batch): the ids
        // an entry load needs are then older than the entries in flight, and
        // no wait drains the queue (vmcnt counts in issue order)
        auto ldid = [&](uint32_t j0, uint32_t* v) {
#pragma unroll
            for (int q = 0; q < kCB; q++) v[q] = vrls[begin + min(j0 + (uint32_t)q, m - 1)];
        };
        auto ldx = [&](const uint32_t* v, float (*x)[kCB]) {
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
#pragma unroll
                for (int q = 0; q < kCB; q++) x[rb][q] = ldg2(Rt, row[rb].base + (size_t)v[q] * row[rb].stride).x;
        };
        auto reduce = [&](uint32_t j0, const uint32_t* v, float (*x)[kCB]) {
            float pn[kCB], pp[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) { pn[q] = 0.0f; pp[q] = 0.0f; }
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
                if (lane + 64u * rb < R) {
#pragma unroll
                    for (int q = 0; q < kCB; q++) { const float a = fabsf(x[rb][q]); pn[q] = pn[q] + a * a; }
                }
            tree_fn<kCB>(pn);
            float nc[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) nc[q] = sqrtf(__shfl(pn[q], 0, 64));
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
                if (lane + 64u * rb < R) {
#pragma unroll
                    for (int q = 0; q < kCB; q++) pp[q] = pp[q] + d[rb] * (x[rb][q] / nc[q]);
                }
            tree_fn<kCB>(pp);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < kCB; q++)
                    if (j0 + q < m) k0[j0 + q] = proj_key(nc[q] != 0 ? pp[q] : 0.0f, v[q]);
            }
        };
        uint32_t j0 = (uint32_t)wave * kCB;
        if (j0 < m) {
            const uint32_t jl = j0 + ((m - 1 - j0) / stride) * stride;   // the wave's last batch
            auto cl = [&](uint32_t j) { return min(j, jl); };
            uint32_t kA[kCB], kB[kCB], vN[kCB];
            float xA[kRB][kCB], xB[kRB][kCB];
            ldid(j0, vN);
#pragma unroll
            for (int q = 0; q < kCB; q++) kA[q] = vN[q];
            ldid(cl(j0 + stride), vN);
            ldx(kA, xA);
            for (;; j0 += 2 * stride) {
#pragma unroll
                for (int q = 0; q < kCB; q++) kB[q] = vN[q];
                ldid(cl(j0 + 2 * stride), vN);
                ldx(kB, xB);
                reduce(j0, kA, xA);
                if (j0 + stride >= m) break;
#pragma unroll
                for (int q = 0; q < kCB; q++) kA[q] = vN[q];
                ldid(cl(j0 + 3 * stride), vN);
                ldx(kA, xA);
                reduce(j0 + stride, kB, xB);
                if (j0 + 2 * stride >= m) break;
            }
        }
    } else {                                // tall local matrices: two passes from memory
        for (uint32_t j0 = (uint32_t)wave * kCB; j0 < m; j0 += stride) {
            uint32_t vr[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) vr[q] = vrls[begin + min(j0 + (uint32_t)q, m - 1)];
            float pn[kCB], pp[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) { pn[q] = 0.0f; pp[q] = 0.0f; }
            for (uint32_t r = lane; r < R; r += 64) {
                const RowRef rw = row_ref(J, r);
#pragma unroll
                for (int q = 0; q < kCB; q++) { const float a = fabsf(ldg2(Rt, rw.base + (size_t)vr[q] * rw.stride).x); pn[q] = pn[q] + a * a; }
            }
            float nc[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) nc[q] = sqrtf(__shfl(tree_f(pn[q]), 0, 64));
            for (uint32_t r = lane; r < R; r += 64) {
                const RowRef rw = row_ref(J, r);
                const float dd = dir[r];
#pragma unroll
                for (int q = 0; q < kCB; q++) pp[q] = pp[q] + dd * (ldg2(Rt, rw.base + (size_t)vr[q] * rw.stride).x / nc[q]);
            }
#pragma unroll
            for (int q = 0; q < kCB; q++) {
                const float pr = tree_f(pp[q]);
                if (lane == 0 && j0 + q < m) k0[j0 + q] = proj_key(nc[q] != 0 ? pr : 0.0f, vr[q]);
            }
        }
    }
}


// The end of a split (:664-684): the argmin over the split position of the
// four prefix variances pref(k, i) (fsu, fsi of the forward pass, feu, fei of
// the reverse one), then the two children pushed (commit) or the result
// written to *res for the leader (sc1 stores, see split()'s range copy).
template <class Pref>
__device__ __forceinline__ void split_finish(CJ& J, Ctl& C, uint32_t begin, uint32_t end, bool commit,
                                             SplitRes* res, Pref pref, uint32_t v_first = 0u, uint32_t v_last = 0u)
{
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t m = end - begin;
    auto& Cs = *lp(&C);
    float bv = INFINITY;
    uint32_t bi = 0xFFFFFFFFu;
    for (uint32_t i = 1 + tid; i < m; i += kThreads) {
        const float v = pref(0, i - 1) + pref(1, i - 1) + pref(2, m - 1 - i) + pref(3, m - 1 - i);
        if (v < bv) { bv = v; bi = i; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_down(bv, off, 64);
        const uint32_t oi = __shfl_down(bi, off, 64);
        if (lane < off && (ov < bv || (ov == bv && oi < bi))) { bv = ov; bi = oi; }
    }
    if (lane == 0) { Cs.best_v[wave] = bv; Cs.best_i[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
        float v = INFINITY;
        uint32_t idx = 0xFFFFFFFFu;
        for (int w = 0; w < kWaves; w++)
            if (Cs.best_v[w] < v || (Cs.best_v[w] == v && Cs.best_i[w] < idx)) { v = Cs.best_v[w]; idx = Cs.best_i[w]; }
        if (!commit) {
            SplitRes r{idx, Cs.err | (idx == 0xFFFFFFFFu ? 1 : 0), 0.0f, 0.0f, 0.0f, 0.0f, v_first, v_last};
            if (idx != 0xFFFFFFFFu) {
                r.fsu = pref(0, idx - 1); r.fsi = pref(1, idx - 1);
                r.feu = pref(2, m - 1 - idx); r.fei = pref(3, m - 1 - idx);
            }
            auto* const rw = gpw(reinterpret_cast<uint32_t*>(res));   // sc1 stores, see split()'s range copy
            const uint32_t* rv = reinterpret_cast<const uint32_t*>(&r);
#pragma unroll
            for (int k = 0; k < (int)(sizeof(SplitRes) / 4); k++)
                __hip_atomic_store(&rw[k], rv[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (idx == 0xFFFFFFFFu) {
            Cs.err = 1;
        } else {
            const uint32_t s = begin + idx;
            add_cluster(J, C, begin, s, pref(0, idx - 1), pref(1, idx - 1));
            add_cluster(J, C, s, end, pref(2, m - 1 - idx), pref(3, m - 1 - idx));
        }
    }
    __syncthreads();
}

// ------------------------------------------------------- fused split --
// A small split whose cluster fits the LDS pool: split() with
// variance_split_small in one function, every phase from LDS.  One pass over
// HBM stages the cluster's m x R entries (float2, [cluster position][row]),
// ids and weights, while wave 0 draws the two centres.  The centres' norms,
// the direction, the projections, the sort (a rank count over the unique
// keys: any correct sort gives std::sort's order), both variance passes and
// the argmin then run without a call or another global round trip; the
// sorted ids and the result are the only stores.  split() reads the entries
// three times from HBM, with about ten dependent round trips and four calls
// per split: the ~50k-cycle floor of a split of a few columns.
// Every value is formed by the same IEEE operations in the same order as
// split() with variance_split_small, so the results are bit-identical.
constexpr uint32_t kFusedMaxRows = 256;
#ifndef ALVRL_FUSED_KB
#define ALVRL_FUSED_KB 16   // staging loads in flight per thread
#endif
// LDS bytes.  XO = false: coefficients 112m, block totals 128m, then the
// entries, 8mR (float2).  XO = true (a cluster whose float2 entries do not
// fit): the entries' means only, 4mR, in the space the coefficients and block
// totals take once the projections are done; the variance passes stream the
// entries from global memory (L2-warm: this workgroup just read them).  Then
// keys 8m, row bases 8R, prefix variances 16m, weights / ids / sorted
// positions / sorted ids 4m each, direction and row strides 4R each.
template <bool XO>
__host__ __device__ constexpr uint32_t fused_base(uint32_t m, uint32_t R)
{
    return XO ? (((4u * m * R > 240u * m ? 4u * m * R : 240u * m) + 7u) & ~7u) : 240u * m + 8u * m * R;
}
template <bool XO>
__host__ __device__ constexpr uint32_t fused_bytes(uint32_t m, uint32_t R)
{
    return fused_base<XO>(m, R) + 40u * m + 16u * R;
}
template <bool XO>
__device__ __forceinline__ bool fused_fits(uint32_t m, uint32_t R)
{
    return m <= kSmallMax && R <= kFusedMaxRows && fused_bytes<XO>(m, R) <= kPoolBytes;
}
__device__ __forceinline__ float readlane0_f(float x)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
}
template <bool XO>
__device__ ALVRL_FUSED_INL void split_fused(CJ& J_in, CC& cm_in, Ctl& C, uint32_t begin, uint32_t end,
                                         unsigned long long* lds, Prof& pf, bool commit, SplitRes* res)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    // uniform in SGPRs: the loops and guards on m branch on scalars
    begin = (uint32_t)__builtin_amdgcn_readfirstlane((int)begin);
    end = (uint32_t)__builtin_amdgcn_readfirstlane((int)end);
    const int tid = threadIdx.x, wave = tid >> 6;
    // the phase profile through typed LDS and global accesses: a flat one
    // (Prof::mark's) makes every later wait of the function a wait for all
    // loads in flight
    auto* const pfs = lp(&pf);
    auto* const pfp = gpw(pfs->p);
    auto padd = [&](int id, unsigned long long v) {
        __hip_atomic_fetch_add(&pfp[id], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto pmark = [&](int id) {
        if (pfp && tid == 0) {
            const long long now = clock64();
            padd(id, (unsigned long long)(now - pfs->t));
            if (pfs->sm >= 0 && id >= PF_WSAMP && id <= PF_ARGMIN)
                padd(kPfSmallAt + pfs->sm * kPfSmallPh + (id - PF_WSAMP), (unsigned long long)(now - pfs->t));
            pfs->t = now;
        }
    };
    pmark(PF_CTRL);
    if (pfp && tid == 0) {
        padd(PF_NSPLIT, 1);
        padd(PF_SPLITCOLS, end - begin);
        pfs->sm = end - begin < 64 ? 0 : end - begin < 256 ? 1 : -1;
    }
    const long long hb0 = pfs->t;
    long long hbv = 0, hbp = 0;
    const uint32_t lane = (uint32_t)(tid & 63);
    const uint32_t m = end - begin, R = J.nrows, NB = (R + 63) / 64;
    auto& Cs = *lp(&C);
    if (!LDS_OK(fused_fits<XO>(m, R), "fused split size", m, R)) return;
    // register copies of the job's fields (see split())
    const auto* const vrlsR = gp(J.vrls);
    auto* const vrlsW = gpw(J.vrls);
    const auto* const colwR = gp(J.colw);
    const uint32_t stage = J.stage_refine;
    const uint32_t seed = cm.seed, pass = cm.pass;
    const float2* const Rt = cm.Rt;
    const int contig = J.contig;
    const unsigned long long off0 = J.off0;
    const uint32_t stride0 = J.stride0;
    unsigned char* const pool = reinterpret_cast<unsigned char*>(lds);
    const uint32_t oE = XO ? 0u : 240u * m, oK = fused_base<XO>(m, R), o4 = oK + 8u * m + 8u * R;
    auto* const coef = lp(reinterpret_cast<double*>(pool));                                // [g][7][m]
    auto* const Q = lp(reinterpret_cast<double*>(pool + 112u * m));                        // [g][c][h][block]
    auto* const Eu = lp(reinterpret_cast<unsigned long long*>(pool + oE));                 // [m][R] (float2 bits; !XO)
    auto* const Ex = lp(reinterpret_cast<float*>(pool + oE));                              // the means
    auto xat = [&](uint32_t i) -> float { return Ex[XO ? i : 2u * i]; };                  // mean of element i = c * R + r
    auto* const keys = lp(reinterpret_cast<unsigned long long*>(pool + oK));               // [m]
    auto* const rbase = lp(reinterpret_cast<unsigned long long*>(pool + oK + 8u * m));     // [R]
    auto* const out = lp(reinterpret_cast<float*>(pool + o4));                             // [4][m]
    float* const wv = reinterpret_cast<float*>(pool + o4 + 16u * m);                       // [m]
    auto* const ids = lp(reinterpret_cast<uint32_t*>(pool + o4 + 20u * m));                // [m]
    auto* const spos = lp(reinterpret_cast<uint32_t*>(pool + o4 + 24u * m));               // [m]: sorted -> cluster position
    auto* const svrl = lp(reinterpret_cast<uint32_t*>(pool + o4 + 28u * m));               // [m]: sorted ids
    auto* const dir = lp(reinterpret_cast<float*>(pool + o4 + 32u * m));                   // [R]
    auto* const rstr = lp(reinterpret_cast<uint32_t*>(pool + o4 + 32u * m + 4u * R));      // [R]
    // this thread's variance row (wave = pass * 4 + row block), its weight in flight from here
    const int g = wave >> 2;
    const uint32_t blk = (uint32_t)(wave & 3);
    const uint32_t vrow = min(blk * 64u + lane, R - 1);
    const double lw = gp(J.locw)[vrow];

    // ids and weights (:597-602); the row layout of a non-contiguous job
    if (tid < (int)m) {
        const uint32_t v = vrlsR[begin + (uint32_t)tid];
        ids[tid] = v;
        lp(wv)[tid] = colwR[v];
    } else if (!contig && tid >= 256 && (uint32_t)tid - 256u < R) {
        const uint32_t r = (uint32_t)tid - 256u;
        rbase[r] = gp(J.roff)[r];
        rstr[r] = gp(J.rstride)[r];
    }
    __syncthreads();
    if (wave == 0) {
        // the two centres (:597-602), as split()
        Smp smp;
        smp.init(seed, pass, begin, end, stage);
        const WsPick p1 = weighted_sample_wave(wv, nullptr, nullptr, m, smp, 0xFFFFFFFFu, false, true);
        smp.k = p1.k; smp.blk = 0xFFFFFFFFu;   // the same stream from draw p1.k
        const WsPick p2 = weighted_sample_wave(wv, nullptr, nullptr, m, smp, p1.idx, false, true);
        if (lane == 0) {
            if (p1.err | p2.err) Cs.err = 1;
            Cs.fi1 = p1.idx; Cs.fi2 = p2.idx;
            Cs.vrl1 = ids[p1.idx]; Cs.vrl2 = ids[p2.idx]; Cs.draw_k = p2.k;
        }
    } else {
        // the entries on waves 1-7, kCB columns per wave and batch, lanes
        // over the rows (split_projections' loads).  No guards: rows past R
        // load and store row R - 1 again, columns past m column m - 1 (the
        // same values to the same places), so that every load of a batch is
        // in flight together -- a load under a per-lane branch makes the
        // compiler wait for every load in flight where the branch rejoins
        const auto* const R64 = gp(reinterpret_cast<const unsigned long long*>(Rt));
        size_t rbs[kRB], rss[kRB];
        uint32_t rcl[kRB];
#pragma unroll
        for (int rb = 0; rb < kRB; rb++) {
            rcl[rb] = min(lane + 64u * rb, R - 1);
            rbs[rb] = contig ? (size_t)(off0 + rcl[rb]) : (size_t)rbase[rcl[rb]];
            rss[rb] = contig ? (size_t)stride0 : (size_t)rstr[rcl[rb]];
        }
        for (uint32_t j0 = (uint32_t)(wave - 1) * kCB; j0 < m; j0 += (kWaves - 1) * kCB) {
            uint32_t jc[kCB], v[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) { jc[q] = min(j0 + (uint32_t)q, m - 1); v[q] = ids[jc[q]]; }
            unsigned long long x[kRB][kCB];
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
#pragma unroll
                for (int q = 0; q < kCB; q++) x[rb][q] = R64[rbs[rb] + (size_t)v[q] * rss[rb]];
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
#pragma unroll
                for (int q = 0; q < kCB; q++) {
                    const uint32_t i = jc[q] * R + rcl[rb];
                    if (XO) Ex[i] = __uint_as_float((uint32_t)x[rb][q]);
                    else Eu[i] = x[rb][q];
                }
        }
    }
    __syncthreads();
    pmark(PF_WSAMP);
    // |c1|, |c2|, |c2 - c1| (:607-616) and the direction (:617-624), wave 0
    if (wave == 0) {
        const uint32_t i1 = Cs.fi1, i2 = Cs.fi2;
        float p1 = 0.0f, p2 = 0.0f, pd = 0.0f;
        for (uint32_t r = lane; r < R; r += 64) {
            const float a = xat(i1 * R + r), b = xat(i2 * R + r);
            const float d = b - a;
            const float ua = fabsf(a), ub = fabsf(b), ud = fabsf(d);
            p1 = p1 + ua * ua; p2 = p2 + ub * ub; pd = pd + ud * ud;
        }
        p1 = tree_f(p1); p2 = tree_f(p2); pd = tree_f(pd);
        const float n1 = sqrtf(readlane0_f(p1)), n2 = sqrtf(readlane0_f(p2)), dl = sqrtf(readlane0_f(pd));
        const bool degen = !(n1 != 0 && n2 != 0 && dl != 0);
        if (lane == 0) {
            Cs.nrm3[0] = n1; Cs.nrm3[1] = n2; Cs.nrm3[2] = dl;
            Cs.diffLen = dl; Cs.degenerate = degen;
        }
        if (!degen)
            for (uint32_t r = lane; r < R; r += 64) dir[r] = (xat(i2 * R + r) - xat(i1 * R + r)) / dl;
    }
    __syncthreads();
    if (Cs.degenerate) {
        // a random direction (:618-621), as split()
        uint32_t k = Cs.draw_k;
        while (true) {
            for (uint32_t r = tid; r < R; r += kThreads) {
                const float sx = draw_at(seed, pass, begin, end, stage, k + 2 * r);
                const float sy = draw_at(seed, pass, begin, end, stage, k + 2 * r + 1);
                dir[r] = det_std_normal_x(sx, sy);
            }
            __syncthreads();
            if (wave == 0) {
                float p = 0.0f;
                for (uint32_t r = lane; r < R; r += 64) { const float u = fabsf(dir[r]); p = p + u * u; }
                p = tree_f(p);
                if (lane == 0) Cs.nd = sqrtf(p);
            }
            __syncthreads();
            if (Cs.nd != 0) break;
            k += 2 * R;
            if (k > Cs.draw_k + 64u * 2u * R) {   // hang guard, as split()
                if (tid == 0) Cs.err = 1;
                __syncthreads();
                break;
            }
        }
        const float nd = Cs.nd != 0 ? Cs.nd : 1.0f;
        for (uint32_t r = tid; r < R; r += kThreads) dir[r] = dir[r] / nd;
        __syncthreads();
    }
    pmark(PF_DIR);
    hbp = pfs->t - hb0;
    // projections (:625-640): split_projections' arithmetic, kCB columns per wave
    {
        float d[kRB];
#pragma unroll
        for (int rb = 0; rb < kRB; rb++) {
            const uint32_t r = lane + 64u * rb;
            d[rb] = r < R ? dir[r] : 0.0f;
        }
        for (uint32_t j0 = (uint32_t)wave * kCB; j0 < m; j0 += kWaves * kCB) {
            uint32_t v[kCB];
            float x[kRB][kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) {
                const uint32_t jc = min(j0 + (uint32_t)q, m - 1);
                v[q] = ids[jc];
#pragma unroll
                for (int rb = 0; rb < kRB; rb++) {
                    const uint32_t r = lane + 64u * rb;
                    x[rb][q] = 64u * rb < R ? xat(jc * R + (r < R ? r : 0u)) : 0.0f;
                }
            }
            float pn[kCB], pp[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) { pn[q] = 0.0f; pp[q] = 0.0f; }
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
                if (lane + 64u * rb < R) {
#pragma unroll
                    for (int q = 0; q < kCB; q++) { const float a = fabsf(x[rb][q]); pn[q] = pn[q] + a * a; }
                }
            tree_fn<kCB>(pn);
            float nc[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) nc[q] = sqrtf(__shfl(pn[q], 0, 64));
#pragma unroll
            for (int rb = 0; rb < kRB; rb++)
                if (lane + 64u * rb < R) {
#pragma unroll
                    for (int q = 0; q < kCB; q++) pp[q] = pp[q] + d[rb] * (x[rb][q] / nc[q]);
                }
            tree_fn<kCB>(pp);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < kCB; q++)
                    if (j0 + q < m) keys[j0 + q] = proj_key(nc[q] != 0 ? pp[q] : 0.0f, v[q]);
            }
        }
    }
    __syncthreads();
    pmark(PF_PROJ);
    // the sort (:641-648): each key's rank among the m unique keys; the
    // sorted ids to vrls (a speculative split's with sc1 stores, as split())
    if (tid < (int)m) {
        const unsigned long long k = keys[tid];
        uint32_t rank = 0;
#pragma unroll 4
        for (uint32_t j = 0; j < m; j++) rank += keys[j] < k ? 1u : 0u;
        spos[rank] = (uint32_t)tid;
        const uint32_t v = ids[tid];
        svrl[rank] = v;
        if (commit) vrlsW[begin + rank] = v;
        else __hip_atomic_store(&vrlsW[begin + rank], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    pmark(PF_SORT);
    const long long hv0 = pfp && tid == 0 ? (long long)clock64() : 0;
    // variance_split_small from LDS: waves 0 / 4 form the forward / reverse
    // pass's coefficients (chunk_coefs, :1075-1085)
    if (blk == 0) {
        auto* const cg = coef + (size_t)g * 7 * m;
        double W = 0.0;
        for (uint32_t c0 = 0; c0 < m; c0 += 64) {
            const uint32_t c = c0 + lane;
            const bool has = c < m;
            const uint32_t i = has ? c : m - 1;
            const double w = (double)lp(wv)[spos[g == 0 ? i : m - 1 - i]];
            const uint32_t n = min(64u, m - c0);
            double Wo = 0.0, Wn = 0.0;
            for (uint32_t k = 0; k < n; k++) {
                const double wk = readlane_d(w, k);
                const bool me = lane == k;
                Wo = me ? W : Wo;
                W = W + wk;
                Wn = me ? W : Wn;
            }
            if (has) {
                if (!isfinite(w) || w <= 0) Cs.err = 1;
                const double rw = 1.0 / w;
                cg[c] = w;
                cg[m + c] = Wo;
                cg[2 * m + c] = (Wn * Wn) / (Wo * Wo);
                cg[3 * m + c] = (rw + 1.0 / Wo);
                cg[4 * m + c] = rw;
                cg[5 * m + c] = Wn;
                cg[6 * m + c] = 1.0 / Wn;
            }
        }
    }
    __syncthreads();
    // the rows' recurrence (:1086-1106), wave = pass * 4 + row block, and each
    // column's two prefix terms reduced over the block (tree16_transposed)
    if (blk < NB) {
        const bool valid = blk * 64u + lane < R;
        const auto* const cg = coef + (size_t)g * 7 * m;
        double sum = 0.0, M = 0.0, V = 0.0;
        const size_t rb0 = contig ? (size_t)(off0 + vrow) : (size_t)rbase[vrow];
        const size_t rs0 = contig ? (size_t)stride0 : (size_t)rstr[vrow];
        auto ld = [&](uint32_t c0, float2* e) {   // XO: from global memory, two chunks ahead
#pragma unroll
            for (int q = 0; q < kCH; q++) {
                const uint32_t c = min(c0 + (uint32_t)q, m - 1), cp = g == 0 ? c : m - 1 - c;
                if (XO) {
                    e[q] = ldg2(Rt, rb0 + (size_t)svrl[cp] * rs0);
                } else {
                    const unsigned long long u = Eu[spos[cp] * R + vrow];
                    e[q] = make_float2(__uint_as_float((uint32_t)u), __uint_as_float((uint32_t)(u >> 32)));
                }
            }
        };
        auto chunk = [&](uint32_t c0, const float2* cur) {
            double tv[2 * kCH];
            if (c0 > 0 && c0 + kCH <= m) {             // a full chunk past column 0: no guards
#pragma unroll
                for (int q = 0; q < kCH; q++) {
                    const uint32_t c = c0 + (uint32_t)q;
                    const double x = (double)cur[q].x;
                    const double tmp = cg[c] * sum - cg[m + c] * x;
                    M = cg[2 * m + c] * M + cg[3 * m + c] * (tmp * tmp);
                    V = V + (double)cur[q].y * cg[4 * m + c];
                    sum = sum + x;
                    tv[2 * q] = lw * (M * cg[6 * m + c]);
                    tv[2 * q + 1] = lw * (V * cg[5 * m + c]);
                }
            } else {
#pragma unroll
                for (int q = 0; q < kCH; q++) {
                    const uint32_t c = c0 + (uint32_t)q;
                    if (c < m) {
                        const double x = (double)cur[q].x;
                        const double tmp = cg[c] * sum - cg[m + c] * x;
                        if (c > 0) M = cg[2 * m + c] * M + cg[3 * m + c] * (tmp * tmp);
                        V = V + (double)cur[q].y * cg[4 * m + c];
                        sum = sum + x;
                        tv[2 * q] = lw * (M * cg[6 * m + c]);
                        tv[2 * q + 1] = lw * (V * cg[5 * m + c]);
                    } else {
                        tv[2 * q] = 0.0; tv[2 * q + 1] = 0.0;
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 2 * kCH; i++) tv[i] = valid ? tv[i] : 0.0;
            const double z = tree16_transposed(tv, lane);
            if ((lane & 3) == 0) {
                const uint32_t h = lane >> 5, c = 4 * ((lane >> 2) & 1) + 2 * ((lane >> 3) & 1) + ((lane >> 4) & 1);
                if (c0 + c < m) Q[(((size_t)g * m + c0 + c) * 2 + h) * 4 + blk] = z;
            }
        };
        // three chunks' entries issued together (clamped: past the end the
        // last chunk again), then the three chunks: nothing is in flight
        // across the loop's back edge, where the compiler would wait for
        // every load (it cannot match loads in flight from two paths)
        const uint32_t nch = (m + kCH - 1) / kCH;
        float2 bufA[kCH], bufB[kCH], bufC[kCH];
        for (uint32_t k = 0; k < nch; k += 3) {
            ld(k * kCH, bufA);
            ld(min(k + 1, nch - 1) * kCH, bufB);
            ld(min(k + 2, nch - 1) * kCH, bufC);
            chunk(k * kCH, bufA);
            if (k + 1 < nch) chunk((k + 1) * kCH, bufB);
            if (k + 2 < nch) chunk((k + 2) * kCH, bufC);
        }
    }
    __syncthreads();
    // block totals in ascending block order (wsum_blk), as floats
    for (uint32_t t = (uint32_t)tid; t < 4 * m; t += kThreads) {
        const uint32_t gh = t / m, c = t - gh * m, gg = gh >> 1, h = gh & 1;
        const auto* q = Q + (((size_t)gg * m + c) * 2 + h) * 4;
        double acc = q[0];
        for (uint32_t b = 1; b < NB; b++) acc = acc + q[b];
        const float f = (h == 0 && c == 0) ? 0.0f : (float)acc;
        out[gh * m + c] = f;
        if (c == m - 1) {
            if (h == 0) Cs.vg[gg].res_u = f; else Cs.vg[gg].res_i = f;
            if (!isfinite(f) || f < 0) Cs.err = 1;
        }
    }
    __syncthreads();
    if (pfp && tid == 0) hbv = (long long)clock64() - hv0;
    pmark(PF_CVF);
    split_finish(J, C, begin, end, commit, res, [&](int k, uint32_t i) -> float { return out[(uint32_t)k * m + i]; },
                 svrl[0], svrl[m - 1]);
    pmark(PF_ARGMIN);
    if (pfp && tid == 0) {
        pfs->sm = -1;
        const int b = pf_bucket(m);
        padd(PF_N + 4 * b, 1ull);
        padd(PF_N + 4 * b + 1, (unsigned long long)(pfs->t - hb0));
        padd(PF_N + 4 * b + 2, (unsigned long long)hbv);
        padd(PF_N + 4 * b + 3, (unsigned long long)hbp);
    }
}

// ------------------------------------------------------------ split --
// Clustering::split (:590-684), collective.
// commit: push the two children (the leader); otherwise write the result to
// *res (a helper working on J with its own scratch and vrls = team.spec)
#ifdef ALVRL_SPLIT_DISPATCH
// (split() below is the inline dispatcher; ALVRL_SPLIT_NODISPATCH: this body is split())
__device__ __noinline__ void split_big(CJ& J_in, CC& cm_in, Ctl& C, uint32_t begin, uint32_t end,
                                       unsigned long long* lds, Prof& pf, bool commit, SplitRes* res)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
#else
__device__ ALVRL_SPLIT_INL void split(CJ& J_in, CC& cm_in, Ctl& C, uint32_t begin, uint32_t end,
                      unsigned long long* lds, Prof& pf, bool commit = true, SplitRes* res = nullptr)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    if (cm.split_fused && cm.var_small) {
        if (fused_fits<false>(end - begin, J.nrows)) {
            split_fused<false>(J, cm, C, begin, end, lds, pf, commit, res);
            return;
        }
        if (cm.split_fused > 1 && fused_fits<true>(end - begin, J.nrows)) {
            split_fused<true>(J, cm, C, begin, end, lds, pf, commit, res);
            return;
        }
    }
#endif
    pf.mark(PF_CTRL);
    pf.count(PF_NSPLIT, 1);
    pf.count(PF_SPLITCOLS, end - begin);
    pf.sm = end - begin < 64 ? 0 : end - begin < 256 ? 1 : -1;
    const long long hb0 = pf.t;
    long long hbv = 0, hbp = 0;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t m = end - begin;
    const uint32_t R = J.nrows;
    if (m >= 4096) EVLOG(cm, 10, m, begin);
    // register copies of the job's fields and of cm: both sit behind generic
    // pointers, so every field read after a barrier would be a flat reload,
    // and a flat op makes the next LDS wait wait for all loads in flight
    const auto* const vrlsR = gp(J.vrls);
    auto* const vrlsW = gpw(J.vrls);
    const auto* const colwR = gp(J.colw);
    auto* const dirW = gpw(J.dir);
    float* const feiP = J.fei;
    const auto* const fsuR = gp(J.fsu);
    const auto* const fsiR = gp(J.fsi);
    const auto* const feuR = gp(J.feu);
    const auto* const feiR = gp(J.fei);
    const uint32_t stage = J.stage_refine;
    const uint32_t seed = cm.seed, pass = cm.pass;
    const float2* const Rt = cm.Rt;
    const int contig = J.contig;
    const unsigned long long off0 = J.off0;
    const uint32_t stride0 = J.stride0;
    const auto* const roffR = gp(J.roff);
    const auto* const rstrR = gp(J.rstride);
    auto rowref = [&](uint32_t r) {
        return contig ? RowRef{(size_t)(off0 + r), (size_t)stride0} : RowRef{(size_t)roffR[r], (size_t)rstrR[r]};
    };
    auto rmean = [&](RowRef rr, uint32_t v) { return ldg2(Rt, rr.base + (size_t)v * rr.stride).x; };
    auto& Cs = *lp(&C);
    // the two centres (:597-602): weights gathered in parallel into contiguous
    // LDS (or scratch for large clusters), scanned by one lane
    const bool wv_lds = (size_t)m * 4 <= kPoolBytes;
    float* wv = wv_lds ? reinterpret_cast<float*>(lds) : feiP;
    {
        constexpr int B = 8;
        for (uint32_t i0 = (uint32_t)tid; i0 < m; i0 += B * kThreads) {
            uint32_t v[B];
#pragma unroll
            for (int b = 0; b < B; b++) v[b] = vrlsR[begin + min(i0 + (uint32_t)b * kThreads, m - 1)];
            float x[B];
#pragma unroll
            for (int b = 0; b < B; b++) x[b] = colwR[v[b]];
#pragma unroll
            for (int b = 0; b < B; b++)
                if (i0 + (uint32_t)b * kThreads < m) {
                    if (wv_lds) lp(wv)[i0 + (uint32_t)b * kThreads] = x[b];
                    else gpw(wv)[i0 + (uint32_t)b * kThreads] = x[b];
                }
        }
    }
    __syncthreads();
    // large clusters: the block totals on every wave (weighted_sample_wg),
    // their LDS array after the weights
    const uint32_t tot_off = wv_lds ? ((m * 4u + 15u) & ~15u) : 0u;
    if (m >= cm.ws_wg_min && tot_off + (m + 63) / 64 * 4u <= kPoolBytes) {
        float* const totp = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(lds) + tot_off);
        Smp smp;
        smp.init(seed, pass, begin, end, stage);
        const WsPick p1 = weighted_sample_wg(wv, wv_lds, m, smp, 0xFFFFFFFFu, totp);
        smp.k = p1.k; smp.blk = 0xFFFFFFFFu;   // the same stream from draw p1.k
        const WsPick p2 = weighted_sample_wg(wv, wv_lds, m, smp, p1.idx, totp);   // colw[vrl1] = 0
        if (tid == 0) {
            if (p1.err | p2.err) Cs.err = 1;
            Cs.vrl1 = vrlsR[begin + p1.idx]; Cs.vrl2 = vrlsR[begin + p2.idx]; Cs.draw_k = p2.k;
        }
    } else if (wave == 0) {
        Smp smp;
        smp.init(seed, pass, begin, end, stage);
        const WsPick p1 = weighted_sample_wave(wv, nullptr, nullptr, m, smp, 0xFFFFFFFFu, false, wv_lds);
        smp.k = p1.k; smp.blk = 0xFFFFFFFFu;   // the same stream from draw p1.k
        const WsPick p2 = weighted_sample_wave(wv, nullptr, nullptr, m, smp, p1.idx, false, wv_lds);   // colw[vrl1] = 0
        const uint32_t i1 = p1.idx, i2 = p2.idx;
        if (lane == 0) {
            if (p1.err | p2.err) Cs.err = 1;
            Cs.vrl1 = vrlsR[begin + i1]; Cs.vrl2 = vrlsR[begin + i2]; Cs.draw_k = p2.k;
        }
    }
    __syncthreads();
    pf.mark(PF_WSAMP);
    if (m >= 4096) EVLOG(cm, 11, m, begin);
    const uint32_t vrl1 = Cs.vrl1, vrl2 = Cs.vrl2;
    // |c1|, |c2|, |c2 - c1| (:607-616), rows in the shared order
    if (wave == 0) {
        float p1 = 0.0f, p2 = 0.0f, pd = 0.0f;
        for (uint32_t r = lane; r < R; r += 64) {
            const RowRef rr = rowref(r);
            const float a = rmean(rr, vrl1), b = rmean(rr, vrl2);
            const float d = b - a;
            const float ua = fabsf(a), ub = fabsf(b), ud = fabsf(d);
            p1 = p1 + ua * ua; p2 = p2 + ub * ub; pd = pd + ud * ud;
        }
        p1 = tree_f(p1); p2 = tree_f(p2); pd = tree_f(pd);
        if (lane == 0) { Cs.nrm3[0] = sqrtf(p1); Cs.nrm3[1] = sqrtf(p2); Cs.nrm3[2] = sqrtf(pd); }
    }
    __syncthreads();
    if (tid == 0) {
        Cs.diffLen = Cs.nrm3[2];
        Cs.degenerate = !(Cs.nrm3[0] != 0 && Cs.nrm3[1] != 0 && Cs.nrm3[2] != 0);
    }
    __syncthreads();
    if (!Cs.degenerate) {
        const float dl = Cs.diffLen;
        for (uint32_t r = tid; r < R; r += kThreads) {
            const RowRef rr = rowref(r);
            const float a = rmean(rr, vrl1), b = rmean(rr, vrl2);
            dirW[r] = (b - a) / dl;
        }
        __syncthreads();
    } else {
        uint32_t k = Cs.draw_k;
        while (true) {
            for (uint32_t r = tid; r < R; r += kThreads) {
                const float sx = draw_at(seed, pass, begin, end, stage, k + 2 * r);
                const float sy = draw_at(seed, pass, begin, end, stage, k + 2 * r + 1);
                dirW[r] = det_std_normal_x(sx, sy);
            }
            __syncthreads();
            if (wave == 0) {
                float p = 0.0f;
                for (uint32_t r = lane; r < R; r += 64) { const float u = fabsf(dirW[r]); p = p + u * u; }
                p = tree_f(p);
                if (lane == 0) Cs.nd = sqrtf(p);
            }
            __syncthreads();
            if (Cs.nd != 0) break;
            k += 2 * R;
            if (k > Cs.draw_k + 64u * 2u * R) {   // hang guard (p ~ 2^-23 per retry)
                if (tid == 0) Cs.err = 1;
                __syncthreads();
                break;
            }
        }
        const float nd = Cs.nd != 0 ? Cs.nd : 1.0f;
        for (uint32_t r = tid; r < R; r += kThreads) dirW[r] = dirW[r] / nd;
        __syncthreads();
    }
    pf.mark(PF_DIR);
    if (m >= 4096) EVLOG(cm, 12, m, begin);
    hbp = pf.t - hb0;
    if (!(cm.parts && cm.proj_min && m >= cm.proj_min && (R > 256 ? cm.part_min_tall : cm.part_min) &&
          proj_parts(J, cm, C, begin, m, reinterpret_cast<unsigned char*>(lds))))
        split_projections(J, cm, begin, m);
    __syncthreads();
    pf.mark(PF_PROJ);
    if (m >= 4096) EVLOG(cm, 13, m, begin);
    const unsigned long long* sorted = sort_keys(J, C, m, lds, cm.sort_radix_min);
    // a speculative split's range and result are handed to the leader, which
    // reads them with agent-scope loads and no acquire (MI355X_MICROARCH.md,
    // valid forms: every store of the handed-off bytes sc1 and drained before
    // the flag, every load of them sc1): agent-scope (sc1) stores here
    if (commit) {
        for (uint32_t i = tid; i < m; i += kThreads) vrlsW[begin + i] = (uint32_t)gp(sorted)[i];
    } else {
        for (uint32_t i = tid; i < m; i += kThreads)
            __hip_atomic_store(&vrlsW[begin + i], (uint32_t)gp(sorted)[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    pf.mark(PF_SORT);
    if (m >= 4096) EVLOG(cm, 14, m, begin);
    const long long hv0 = pf.p && tid == 0 ? (long long)clock64() : 0;
    const bool small = cm.var_small && m <= kSmallMax && R <= 64u * kSmallBlocks;
    unsigned char* const pool = reinterpret_cast<unsigned char*>(lds);
    if (small)
        variance_split_small(J, cm, C, J.vrls + begin, m, pool);
    else
        variance_passes(J, cm, C, J.vrls + begin, m, 2, J.fsu, J.fsi, J.feu, J.fei, pool, &pf);
    if (pf.p && tid == 0) hbv = (long long)clock64() - hv0;
    pf.mark(PF_CVF);
    if (m >= 4096) EVLOG(cm, 15, m, begin);
    // the prefix variances: fsu/fsi of the forward pass, feu/fei of the reverse
    const auto* const so = lp(small_out(pool));
    auto pref = [&](int k, uint32_t i) -> float {
        if (small) return so[k * kSmallMax + i];
        return k == 0 ? fsuR[i] : k == 1 ? fsiR[i] : k == 2 ? feuR[i] : feiR[i];
    };
    // argmin over split position (:664-675), the children or the result
    uint32_t v_first = 0u, v_last = 0u;
    if (!commit && tid == 0) { v_first = (uint32_t)gp(sorted)[0]; v_last = (uint32_t)gp(sorted)[m - 1]; }
    split_finish(J, C, begin, end, commit, res, pref, v_first, v_last);
    pf.mark(PF_ARGMIN);
    if (m >= 4096) EVLOG(cm, 16, m, begin);
    pf.sm = -1;
    if (pf.p && tid == 0) {
        const int b = pf_bucket(m);
        gadd(&pf.p[PF_N + 4 * b], 1ull);
        gadd(&pf.p[PF_N + 4 * b + 1], (unsigned long long)(pf.t - hb0));
        gadd(&pf.p[PF_N + 4 * b + 2], (unsigned long long)hbv);
        gadd(&pf.p[PF_N + 4 * b + 3], (unsigned long long)hbp);
    }
}
#ifdef ALVRL_SPLIT_DISPATCH
__device__ __forceinline__ void split(CJ& J_in, CC& cm_in, Ctl& C, uint32_t begin, uint32_t end,
                                      unsigned long long* lds, Prof& pf, bool commit = true, SplitRes* res = nullptr)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    if (cm.split_fused && cm.var_small) {
        if (fused_fits<false>(end - begin, J.nrows)) {
            split_fused<false>(J, cm, C, begin, end, lds, pf, commit, res);
            return;
        }
        if (cm.split_fused > 1 && fused_fits<true>(end - begin, J.nrows)) {
            split_fused<true>(J, cm, C, begin, end, lds, pf, commit, res);
            return;
        }
    }
    split_big(J, cm, C, begin, end, lds, pf, commit, res);
}
#endif

// ------------------------------------------------------- team mode --
__device__ __forceinline__ unsigned long long ld_acq(unsigned long long* p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_acq(uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ bool cas_acq_rel(T* p, T expect, T v)
{
    return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
// Polling uses relaxed agent-scope loads (coherent across XCDs without
// invalidating the L2 on every iteration); one acquire fence follows success.
__device__ __forceinline__ unsigned long long ld_rlx(unsigned long long* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_rlx(uint32_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fence_acq() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }
// Task bookkeeping (queue slots, tail, head, per-cluster state words) carries
// no payload of its own: relaxed agent-scope atomics, ordered where it
// matters by draining them (s_waitcnt vmcnt(0)) before the next one.  The
// only payload is the vrls a helper copies, released once per split by the
// leader (split_team) and acquired by the helper (spec_split).  An
// agent-scope release is an L2 write-back (MI355X_MICROARCH.md, fence table).
__device__ __forceinline__ void st_rlx(unsigned long long* p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(uint32_t* p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ bool cas_rlx(T* p, T expect, T v)
{
    return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// constant 100 MHz clock.  No wait is unbounded: a leader that has waited
// Common::wait_ticks (default kSpinTicks, ~60 s) for a helper retires its
// job's team (split_team: stop flag, and every later split of the job is the
// leader's own, so nothing the late helper writes to team.spec / team.res /
// team.state is read again), an idle helper gives up after spin_ticks
// without a task.
__device__ __forceinline__ unsigned long long wall() { return __builtin_amdgcn_s_memrealtime(); }
// thread 0: trace point k of the current pop (ALVRL_POP_TRACE)
__device__ __forceinline__ void pmark(const Ctl& C, int k)
{
    if (threadIdx.x == 0 && C.prec) gpw(C.prec)[k] = (uint32_t)wall();
}
constexpr unsigned long long kSpinTicks = 6000000000ull;   // default of Common::spin_ticks

// Thread 0 of the leader: queue the multi-clusters near the top of the heap
// that are not queued yet.
// The leader's queueing of the clusters near the top of the heap, on wave 0:
// lane k examines heap entries k, k + 64 (one round trip per 64 instead of a
// dependent chain on lane 0); the first 'room' eligible entries in heap order
// are queued, as the sequential loop would.  The vrls of every cluster in the
// heap were released when its parent's split ended (split_team).
template <int PL = -1>
__device__ void enqueue_candidates(CJ& J_in, CC& cm_in, Ctl& C)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    CT& T = J.team;
    const uint32_t lane = threadIdx.x & 63;
    // the heap's first Kt entries, 64 per round (lane = entry), in heap order
    const int Kt = min(min(C.heap_n, (int)(cm.spec_width ? cm.spec_width : 2 * T.helpers + 2)), kSpecWidthMax);
    const HeapRef H = heap_of(J, C);
    const uint32_t tail = C.qtail;
    uint32_t head = C.qhead, npush = 0, room = 0;
    for (int base = 0; base < Kt; base += 64) {
        const int K = min(Kt - base, 64);
        bool elig = false;
        uint32_t flags = 0u;
        CNode cn{0.0f, 0.0f, 0u, 0u};
        if ((int)lane < K) {
            cn = hld<PL>(H, base + (int)lane);
            flags = cn.end & ~kEndMask;
            cn.end &= kEndMask;
            elig = cn.end - cn.begin >= cm.spec_min && !(flags & kEndQ);   // not queued by this leader yet
        }
        const unsigned long long bal = __ballot(elig);
        const uint32_t want = (uint32_t)__popcll(bal);
        if (base == 0) {
            // room from the head seen last (helpers only advance it); reloaded when short
            if (want && tail - head + want > kQueue) head = ld_rlx(&T.ctl[0]);
            const uint32_t used = tail - head;
            room = used >= kQueue ? 0u : kQueue - used;
        }
        const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const uint32_t rank = (uint32_t)__popcll(bal & lt);
        const bool queued = elig && rank < room;
        if (queued) {
            const bool spec = (flags & kEndS) != 0;
            st_rlx(&T.state[cn.begin], ((unsigned long long)cn.end << 3) | kStQueued | (spec ? kStSpecBit : 0ull));
            st_rlx(&T.queue[(tail + npush + rank) % kQueue], ((unsigned long long)cn.begin << 32) | cn.end | (spec ? kQSpecBit : 0u));
            hst<PL>(H, base + (int)lane, CNode{cn.uvar, cn.ivar, cn.begin, cn.end | flags | kEndQ});   // (a flag: not logged)
            tcount(cm, TS_ENQ);
        }
        const uint32_t n = min(want, room);
        npush += n;
        room -= n;
    }
    if (lane == 0) {
        C.qhead = head;
        C.pre_b = ~0u;
        // the slots are published with the next split_team's first look
        // (publish_tail), by when these stores have landed
        if (npush) { C.qtail = tail + npush; C.qpend = 1; }
    }
}

// Thread 0 of the leader: publish the slots enqueue_candidates wrote (their
// stores land before the tail that publishes them).
__device__ __forceinline__ void publish_tail(CT& T, Ctl& C)
{
    if (C.qpend) {
        drain_vmem();
        st_rlx(&T.ctl[1], C.qtail);
        C.qpend = 0;
    }
}

// Thread 0 of the leader: queue [b, e) ahead of the heap (the first initial
// cluster, the root of the refinement, while the leader is still computing
// the initial clusters' variances).  Its vrls and the column weights were
// released by the caller.  Popped later, the cluster is stolen back, waited
// for or committed exactly like a cluster enqueue_candidates queued.
__device__ void enqueue_early(CJ& J_in, CC& cm_in, Ctl& C, uint32_t b, uint32_t e)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    CT& T = J.team;
    if (e <= b || e - b < cm.spec_min) return;
    const uint32_t tail = C.qtail;   // (the first enqueue: nothing pending)
    if (tail - ld_rlx(&T.ctl[0]) >= kQueue) return;
    st_rlx(&T.state[b], ((unsigned long long)e << 3) | kStQueued);
    st_rlx(&T.queue[tail % kQueue], ((unsigned long long)b << 32) | e);
    tcount(cm, TS_ENQ);
    drain_vmem();   // slot and state land before the tail that publishes them
    st_rlx(&T.ctl[1], tail + 1);
    C.qtail = tail + 1;
    C.early_b = b;   // its heap node is flagged queued when the leader adds it
}

__device__ void stop_team(CJ& J_in, CC& cm_in, Ctl& C)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    if (J.team.helpers && threadIdx.x == 0) { publish_tail(J.team, C); st_rel(&J.team.ctl[2], 1u); }
    trace(cm, 6, 0);
}

// Block copy of vrls[b, e) between the job's array and the side buffer:
// typed global accesses, eight loads in flight per thread before their
// stores (a one-element loop waits out a cross-XCD load per element).
__device__ void copy_range(uint32_t* dst, const uint32_t* src, uint32_t b, uint32_t e)
{
    const auto d = gpw(dst);
    const auto sp = gp(src);
    constexpr uint32_t U = 8;
    for (uint32_t i0 = b + threadIdx.x; i0 < e; i0 += U * kThreads) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t k = 0; k < U; k++) {
            const uint32_t i = i0 + k * kThreads;
            v[k] = i < e ? sp[i] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < U; k++) {
            const uint32_t i = i0 + k * kThreads;
            if (i < e) d[i] = v[k];
        }
    }
}

// copy_range with agent-scope (sc1) loads: the leader's commit of a result a
// helper stored with sc1 stores (split), read without an acquire
__device__ void copy_range_sc1(uint32_t* dst, const uint32_t* src, uint32_t b, uint32_t e)
{
    const auto d = gpw(dst);
    const auto sp = gp(src);
    constexpr uint32_t U = 8;
    for (uint32_t i0 = b + threadIdx.x; i0 < e; i0 += U * kThreads) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t k = 0; k < U; k++) {
            const uint32_t i = i0 + k * kThreads;
            v[k] = __hip_atomic_load(&sp[i < e ? i : b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (uint32_t k = 0; k < U; k++) {
            const uint32_t i = i0 + k * kThreads;
            if (i < e) d[i] = v[k];
        }
    }
}

// Workgroup w's view of job j (Common::views): roamers 0.., then the helpers
// of job 0, 1, ..., then the leaders
__device__ __forceinline__ uint32_t wid_helper(CC& cm, uint32_t j, uint32_t hid) { return cm.nroam + j * (cm.team - 1) + hid; }
__device__ __forceinline__ uint32_t wid_leader(CC& cm, uint32_t j) { return cm.nroam + cm.njobs * (cm.team - 1) + j; }
__device__ __forceinline__ CJ& view_of(CC& cm, uint32_t w, uint32_t j) { return uni(cm.views[(size_t)w * cm.njobs + j]); }

// Thread 0: take the oldest queued task.  1 = claimed (*b, *e), 0 = queue
// empty, 2 = lost a race (try again).
__device__ int try_claim(CT& T_in, uint32_t* b, uint32_t* e, uint64_t max_cols = ~0ull)
{
    CT& T = uni(T_in);
    const uint32_t h = ld_rlx(&T.ctl[0]), t = ld_rlx(&T.ctl[1]);
    if (h >= t) return 0;
    const unsigned long long task = ld_rlx(&T.queue[h % kQueue]);
    if (((uint32_t)task & ~kQSpecBit) - (uint32_t)(task >> 32) > max_cols) return 0;
    if (!cas_rlx(&T.ctl[0], h, h + 1)) return 2;
    *b = (uint32_t)(task >> 32); *e = (uint32_t)task;   // end with kQSpecBit
    const unsigned long long key = ((unsigned long long)(*e & ~kQSpecBit) << 3) | ((*e & kQSpecBit) ? kStSpecBit : 0ull);
    return cas_rlx(&T.state[*b], key | kStQueued, key | kStRunning) ? 1 : 2;   // spec_split acquires
}

// ------------------------------------------------------- split parts --
// Thread 0: the next part of slot S (-1: every part is claimed).  The CAS
// reads the generation word the owner stored after its release fence, and
// the acquire fence after it makes the slot's fields (and the owner's cw)
// visible to this CU.
__device__ int part_claim_slot(CC& cm_in, PartSlot* S)
{
    CC& cm = uni(cm_in);
    while (true) {
        const unsigned long long w = ld_rlx(&S->word);
        const uint32_t np = (uint32_t)(w >> 16) & 0xFFFFu, nx = (uint32_t)w & 0xFFFFu;
        if (nx >= np) return -1;
        if (cas_rlx(&S->word, w, w + 1ull)) {
            if (nx + 1 == np) __hip_atomic_fetch_add(cm.part_open, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fence_acq();
            return (int)nx;
        }
    }
}
// Thread 0 of an idle workgroup: claim a part of any open slot.
__device__ bool part_try(CC& cm_in, uint32_t* slot, uint32_t* part)
{
    CC& cm = uni(cm_in);
    if (!cm.parts || ld_rlx(cm.part_open) == 0u) return false;
    for (uint32_t s = 0; s < cm.nslots; s++) {
        const int p = part_claim_slot(cm, &cm.parts[s]);
        if (p >= 0) { *slot = s; *part = (uint32_t)p; return true; }
    }
    return false;
}
template <class JV>
__device__ void colw_raw(const JV& J, CC& cm, Ctl& C, uint32_t vb, uint32_t ve);
// Every thread: run part p of slot s and publish it (spec_split's producer
// form: drained stores, barrier, one agent release, relaxed count).  C.err
// is the caller's.
__device__ __noinline__ void run_part(CC& cm_in, Ctl& C, uint32_t s, uint32_t p, unsigned char* pool, bool own)
{
    CC& cm = uni(cm_in);
    PartSlot* const S = &cm.parts[s];
    if (threadIdx.x == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // thread 0's acquire, complete
    __syncthreads();
    // the part's view in LDS: its readers' field loads are LDS reads, not
    // per-lane flat loads whose waits include every store in flight
    __shared__ PartJob pjs;
    static_assert(sizeof(PartJob) % 4 == 0 && sizeof(PartJob) / 4 <= 64, "PartJob copy");
    if (threadIdx.x < sizeof(PartJob) / 4)   // one dword per lane, typed global loads
        reinterpret_cast<uint32_t*>(&pjs)[threadIdx.x] = gp(reinterpret_cast<const uint32_t*>(&S->pj))[threadIdx.x];
    const double* const T = gp(&S->T)[0];
    const int err_saved = C.err;
    __syncthreads();
    const PartJob& pj = pjs;
    if (threadIdx.x == 0) C.err = 0;
    EVLOG(cm, 30, pj.kind, p);
    __syncthreads();
    if (pj.kind == kPartProj || pj.kind == kPartColw) {
        const uint32_t jb = pj.c0 + p * pj.cpp;
        if (jb < pj.m) {
            if (pj.kind == kPartProj) proj_range(pj, cm, jb, min(pj.m, jb + pj.cpp));
            else colw_raw(pj, cm, C, jb, min(pj.m, jb + pj.cpp));
        }
    } else if (pj.kind == kPartInit) {
        const uint32_t gb0 = p * pj.pblk;
        if (LDS_OK(gb0 < pj.nblk && pj.pblk <= kPartMaxBlk, "part blocks", gb0, pj.nblk))
            variance_part<false>(pj, cm, C, nullptr, 0, gb0, min(pj.pblk, pj.nblk - gb0), pool);
    } else {
        const uint32_t g = p & 1u, gb0 = (p >> 1) * pj.pblk;
        if (LDS_OK(gb0 < pj.nblk && pj.pblk <= kPartMaxBlk, "part blocks", gb0, pj.nblk))
            variance_part<true>(pj, cm, C, T, g, gb0, min(pj.pblk, pj.nblk - gb0), pool);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    EVLOG(cm, 31, pj.kind, pj.m);
    if (threadIdx.x == 0) {
        if (C.err) __hip_atomic_fetch_or(&S->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        C.err = err_saved;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(&S->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tcount(cm, own ? TS_POWN : TS_POTHER);
    }
    __syncthreads();
}
// Every thread: a free slot of the board whose block-total buffer holds a
// split of `cols` columns (0: none needed), or -1.  Slots [0, nbig) hold any
// split, the others up to small_cap columns; small needs try those first.
__device__ int part_slot_take(CC& cm_in, Ctl& C, uint32_t cols, uint32_t rows)
{
    CC& cm = uni(cm_in);
    if (threadIdx.x == 0) {
        int got = -1;
        // too few workgroups idle to take parts: the one-workgroup engines
        const uint32_t imin = rows > 256 ? cm.idle_min : cm.idle_min_short;
        const bool idle = imin == 0 || ld_rlx(cm.idle) >= imin;
        auto scan = [&](uint32_t lo, uint32_t hi) {
            if (hi <= lo) return;
            const uint32_t n = hi - lo;
            uint32_t s = lo + blockIdx.x % n;   // owners spread over the slots
            for (uint32_t i = 0; i < n && got < 0; i++) {
                if (ld_rlx(&cm.parts[s].busy) == 0u && cas_rlx(&cm.parts[s].busy, 0u, 1u)) got = (int)s;
                if (++s == hi) s = lo;
            }
        };
        if (idle && cols <= cm.small_cap) scan(cm.nbig, cm.nslots);
        if (idle && got < 0) scan(0, cm.nbig);
        C.go = got;
        if (got < 0) tcount(cm, TS_PSOLO);
    }
    __syncthreads();
    const int sl = C.go;
    __syncthreads();
    return sl;
}
// Every thread: publish pj's parts on slot sl (its inputs stored by this
// workgroup before the call), run parts until none is left, then wait for
// the claimed ones.  The claimed parts run on workgroups that wait for
// nobody, so the wait ends; a 60 s guard fails the job (false) and keeps the
// slot, which a late part may still write.
__device__ bool part_run_all(CC& cm_in, Ctl& C, uint32_t sl, const PartJob& pj, unsigned char* pool)
{
    CC& cm = uni(cm_in);
    PartSlot* const S = &cm.parts[sl];
    const int tid = threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        S->pj = pj;
        st_rlx(&S->done, 0u);
        st_rlx(&S->err, 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long w = ld_rlx(&S->word);
        st_rlx(&S->word, (((w >> 32) + 1ull) << 32) | ((unsigned long long)pj.np << 16));
        __hip_atomic_fetch_add(cm.part_open, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        tcount(cm, TS_PSPLIT);
    }
    __syncthreads();
    while (true) {
        if (tid == 0) C.go = part_claim_slot(cm, S);
        __syncthreads();
        const int p = C.go;
        __syncthreads();
        if (p < 0) break;
        run_part(cm, C, sl, (uint32_t)p, pool, true);
    }
    if (tid == 0) {
        const unsigned long long t0 = wall();
        int ok = 1;
        while (ld_rlx(&S->done) != pj.np) {
            if (wall() - t0 > kSpinTicks) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(4);
        }
        tadd(cm, TS_PWAIT, wall() - t0);
        fence_acq();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!ok || ld_rlx(&S->err)) C.err = 1;
        C.go = ok;
    }
    __syncthreads();
    const bool ok = C.go != 0;
    __syncthreads();
    return ok;
}
__device__ void part_slot_free(CC& cm_in, uint32_t sl)
{
    CC& cm = uni(cm_in);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&cm.parts[sl].busy, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// Every thread: the cluster's (weight << 32 | vrl) pairs in column order, for
// every part of a divided variance pass (variance_split_v3's gather)
__device__ void gather_cw(CJ& J_in, const uint32_t* base, uint32_t m, unsigned long long* cw)
{
    CJ& J = uni(J_in);
    constexpr int B = 8;
    for (uint32_t i0 = threadIdx.x; i0 < m; i0 += B * kThreads) {
        uint32_t v[B];
#pragma unroll
        for (int b = 0; b < B; b++) v[b] = gp(base)[min(i0 + (uint32_t)b * kThreads, m - 1)];
        float wt[B];
#pragma unroll
        for (int b = 0; b < B; b++) wt[b] = gp(J.colw)[v[b]];
#pragma unroll
        for (int b = 0; b < B; b++)
            if (i0 + (uint32_t)b * kThreads < m)
                gpw(cw)[i0 + (uint32_t)b * kThreads] = ((unsigned long long)__float_as_uint(wt[b]) << 32) | v[b];
    }
}
// The owner's side of a divided split's variance passes (variance_passes,
// both passes with prefixes): false when no slot is free (the caller runs the
// one-workgroup engine).  The cluster's (weight, vrl) pairs are gathered once
// for every part; afterwards the block totals are added in ascending block
// order into the float prefixes (variance_split_v3's reduce, the last group's).
__device__ __noinline__ bool split_parts(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* base, uint32_t m,
                            float* fu0, float* fi0, float* fu1, float* fi1, unsigned char* pool)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int tid = threadIdx.x;
    const int sl = part_slot_take(cm, C, m, J.nrows);
    if (sl < 0) return false;
    unsigned long long* const cw = J.keys1;
    gather_cw(J, base, m, cw);
    EVLOG(cm, 20, m, J.nrows);
    const uint32_t nblk = (J.nrows + 63) / 64,
                   pblk = min(max(J.nrows > 256 ? cm.part_blk : cm.part_blk_short, 1u), kPartMaxBlk);
    PartJob pj = part_job(J);
    pj.kind = kPartVar; pj.cw = cw; pj.m = m; pj.nblk = nblk; pj.pblk = pblk;
    pj.np = 2 * ((nblk + pblk - 1) / pblk);
    if (!part_run_all(cm, C, (uint32_t)sl, pj, pool)) return true;
    EVLOG(cm, 21, m, pj.np);
    const double* const T = gp(&cm.parts[sl].T)[0];
    // the block totals added in block order; up to 4 blocks, 8 sums per
    // thread with all their loads issued before the adds (one round trip)
    auto finish = [&](uint32_t t, double acc) {
        const uint32_t gh = t / m, n = t - gh * m, g = gh >> 1, h = gh & 1;
        const float f = (h == 0 && n == 0) ? 0.0f : (float)acc;
        float* const out = g == 0 ? (h == 0 ? fu0 : fi0) : (h == 0 ? fu1 : fi1);
        gpw(out)[n] = f;
        if (n == m - 1) {
            if (h == 0) C.vg[g].res_u = f; else C.vg[g].res_i = f;
            if (!isfinite(f) || f < 0) C.err = 1;
        }
    };
    const uint32_t tot = 4u * m;
    if (nblk <= 4) {
        constexpr uint32_t U = 8;
        for (uint32_t t0 = (uint32_t)tid; t0 < tot; t0 += U * kThreads) {
            double x[4][U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t t = min(t0 + u * kThreads, tot - 1), gh = t / m, n = t - gh * m;
                const auto* q = gp(T + (size_t)gh * nblk * m + n);
#pragma unroll
                for (uint32_t b = 0; b < 4; b++) x[b][u] = q[(size_t)min(b, nblk - 1) * m];
            }
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                double acc = x[0][u];
#pragma unroll
                for (uint32_t b = 1; b < 4; b++) acc = b < nblk ? acc + x[b][u] : acc;
                if (t0 + u * kThreads < tot) finish(t0 + u * kThreads, acc);
            }
        }
    } else {
        for (uint32_t t = (uint32_t)tid; t < tot; t += kThreads) {
            const uint32_t gh = t / m, n = t - gh * m;
            const auto* q = gp(T + (size_t)gh * nblk * m + n);
            double acc = q[0];
            for (uint32_t b = 1; b < nblk; b++) acc = acc + q[(size_t)b * m];
            finish(t, acc);
        }
    }
    EVLOG(cm, 22, m, 0);
    part_slot_free(cm, (uint32_t)sl);
    return true;
}
// The owner's side of a divided split's projections (split): column ranges
// of the cluster on idle workgroups.  False when no slot is free.
__device__ __noinline__ bool proj_parts(CJ& J_in, CC& cm_in, Ctl& C, uint32_t begin, uint32_t m, unsigned char* pool)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int sl = part_slot_take(cm, C, 0u, J.nrows);
    if (sl < 0) return false;
    PartJob pj = part_job(J);
    pj.kind = kPartProj; pj.ids = J.vrls + begin; pj.dir = J.dir; pj.keys = J.keys0; pj.m = m;
    pj.cpp = max(cm.proj_cpp, 64u);
    pj.np = min((m + pj.cpp - 1) / pj.cpp, 0xFFFFu);
    pj.cpp = (m + pj.np - 1) / pj.np;
    // a timed-out slot stays busy: a late part may still write into it
    // (part_run_all; C.err is set and the job fails)
    if (part_run_all(cm, C, (uint32_t)sl, pj, pool)) part_slot_free(cm, (uint32_t)sl);
    return true;
}
// The owner's side of divided column weights (calculateColumnWeigths over
// columns [vb, ve), each column's sum its own): false when no slot is free.
__device__ __noinline__ bool colw_parts(CJ& J_in, CC& cm_in, Ctl& C, uint32_t vb, uint32_t ve,
                                        unsigned char* pool)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int sl = part_slot_take(cm, C, 0u, J.nrows);
    if (sl < 0) return false;
    PartJob pj = part_job(J);
    pj.kind = kPartColw; pj.colw = J.colw; pj.c0 = vb; pj.m = ve;
    pj.cpp = max(cm.proj_cpp, 64u);
    pj.np = min((ve - vb + pj.cpp - 1) / pj.cpp, 0xFFFFu);
    pj.cpp = (ve - vb + pj.np - 1) / pj.np;
    if (part_run_all(cm, C, (uint32_t)sl, pj, pool)) part_slot_free(cm, (uint32_t)sl);   // as proj_parts
    return true;
}
// The owner's side of a divided cluster variance (variance_passes without
// prefixes, one pass, more than 256 rows): each part writes its rows' final
// states, then wave 0 forms the two sums over all rows as
// variance_split_v3<false>'s last group does.  False when no slot is free.
__device__ __noinline__ bool init_parts(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* base, uint32_t m,
                                        unsigned char* pool)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int sl = part_slot_take(cm, C, 0u, J.nrows);
    if (sl < 0) return false;
    gather_cw(J, base, m, J.keys1);
    // tall jobs: one row block per part (ALVRL_PART_BLK_INIT) -- the setup is
    // every job's critical path and idle workgroups abound then
    const uint32_t nblk = (J.nrows + 63) / 64,
                   pblk = min(max(J.nrows > 256 ? cm.part_blk_init : cm.part_blk_short, 1u), kPartMaxBlk);
    PartJob pj = part_job(J);
    pj.kind = kPartInit; pj.cw = J.keys1; pj.m = m; pj.nblk = nblk; pj.pblk = pblk;
    pj.np = (nblk + pblk - 1) / pblk;
    pj.st = J.st; pj.wsum = &cm.parts[sl].wsum;
    const bool done = part_run_all(cm, C, (uint32_t)sl, pj, pool);
    if (done && threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x, Rfull = J.nrows;
        const double* st = J.st;
        const double Wt = gp(pj.wsum)[0], rW = 1.0 / Wt;
        double pu = 0.0, pi = 0.0;
        for (uint32_t r = lane; r < Rfull; r += 64) {
            pu = pu + J.locw[r] * (gp(st)[Rfull + r] * rW);
            pi = pi + J.locw[r] * (gp(st)[2 * Rfull + r] * Wt);
        }
        pu = tree_d(pu);
        pi = tree_d(pi);
        if (lane == 0) {
            VarGroup& V = C.vg[0];
            V.Wcur = Wt;
            V.res_u = (float)pu; V.res_i = (float)pi;
            if (!isfinite(V.res_u) || V.res_u < 0) C.err = 1;
            if (!isfinite(V.res_i) || V.res_i < 0) C.err = 1;
        }
    }
    if (done) part_slot_free(cm, (uint32_t)sl);   // as proj_parts
    __syncthreads();
    return true;
}

// Split [b, e) speculatively with Jw's scratch (Jw.vrls = team.spec; e may
// carry kQSpecBit: the input is there already) and
// publish the result (MI355X_MICROARCH.md, valid producer form: every storing
// wave drains, barrier, lane 0 releases at agent scope and drains the
// write-back, then the relaxed agent flag store).  C.err is the caller's.
__device__ void spec_split(CJ& J0_in, CJ& Jw_in, CC& cm_in, Ctl& C,
                           unsigned long long* lds, uint32_t b, uint32_t e)
{
    CJ& J0 = uni(J0_in);
    CJ& Jw = uni(Jw_in);
    CC& cm = uni(cm_in);
    CT& T = J0.team;
    const int tid = threadIdx.x;
    const bool in_spec = (e & kQSpecBit) != 0;
    e &= ~kQSpecBit;
    // one agent acquire for the CU (its L1), complete before the barrier
    if (tid < 64) {
        const unsigned long long ta = wall();
        fence_acq();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) tadd(cm, TS_ACQ, wall() - ta);
    }
    __syncthreads();
    if (!in_spec)
        copy_range(T.spec, J0.vrls, b, e);
    __syncthreads();
    const int err_saved = C.err;
    __syncthreads();
    __shared__ Prof off;
    if (tid == 0) { C.err = 0; off.p = nullptr; off.t = 0; off.sm = -1; }
    __syncthreads();
    split(Jw, cm, C, b, e, lds, off, false, &T.res[b]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        C.err = err_saved;
        const unsigned long long tr = wall();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tadd(cm, TS_REL, wall() - tr);
        __hip_atomic_store(&T.state[b], ((unsigned long long)e << 3) | kStDone, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
}

// The commit of a finished speculative split of [b, e) (split_team's mode
// 1).  The result and the range were stored sc1 and drained before the done
// flag (split, spec_split): sc1 loads, no acquire, and no barrier: thread 0
// pushes the children (a single's id from the spec range) while the range
// copy is in flight; wave 0 then queues, and the range's readers come after
// later barriers.
template <int PL = -1>
__device__ __forceinline__ void commit_spec(CJ& J, Ctl& C, uint32_t b, uint32_t e)
{
    CT& T = J.team;
    const int tid = threadIdx.x;
    SplitRes r;
    if (tid == 0) {
        const auto* rr = gp(reinterpret_cast<const uint32_t*>(&T.res[b]));
        uint32_t* rv = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(SplitRes) / 4); k++)
            rv[k] = __hip_atomic_load(&rr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    copy_range_sc1(J.vrls, T.spec, b, e);
    if (tid == 0) {
        if (r.err || r.idx == 0xFFFFFFFFu) {
            C.err = 1;
        } else {
            const uint32_t m = e - b, s2 = b + r.idx;
            add_cluster<PL>(J, C, b, s2, r.fsu, r.fsi, T.spec, 0u, r.v_first);   // a single's id: the result's
            add_cluster<PL>(J, C, s2, e, r.feu, r.fei, T.spec, 0u, r.v_last);
            // the children's input is this result, in team.spec
            st_rlx(&T.state[b], ((unsigned long long)s2 << 3) | kStNone | kStSpecBit);
            st_rlx(&T.state[s2], ((unsigned long long)e << 3) | kStNone | kStSpecBit);
            (void)m;
        }
    }
}

// The leader's usual split (split_team at N >= 2, where the pops are the
// critical path): the popped cluster's speculative split has finished (the
// word pop_wave fetched says done), so the leader commits it and queues the
// next candidates.  Out of line and without calls: it saves no callee-saved
// registers on entry, which split_team (its splits' state lives across calls)
// does on every pop.  commit_ready_ok is uniform (C after the pop's barrier).
__device__ __forceinline__ bool commit_ready_ok(CJ& J, CC& cm, const Ctl& C, uint32_t e)
{
    return J.team.helpers && !C.team_off && !cm.enq_start && !(C.hlds && C.heap_n + 2 > kHeapLdsMax) &&
           (uint32_t)(C.sw >> 3) == e && (C.sw & 7) == kStDone;
}
// (PL: the heap's placement, so that an LDS heap's pushes and queueing do
// not wait for the range copy's stores)
template <int PL>
__device__ __forceinline__ void commit_ready_t(CJ& J, CC& cm, Ctl& C, uint32_t b, uint32_t e)
{
    const int tid = threadIdx.x;
    if (tid == 0) {
        publish_tail(J.team, C);
        trace(cm, 3, b);
        tcount(cm, TS_COMMIT);
        if (C.prec) gpw(C.prec)[7] = 1u | (min(e - b, 0xFFFFFFu) << 8);
    }
#ifndef ALVRL_PT_POP
    pmark(C, 2);
    pmark(C, 3);
#endif
    commit_spec<PL>(J, C, b, e);
#ifndef ALVRL_PT_POP
    pmark(C, 4);
#endif
    if (tid < 64) {
        if (PL == 0) drain_vmem();   // wave 0 queues from the global heap thread 0 just wrote
        enqueue_candidates<PL>(J, cm, C);
    }
    if (tid == 0) trace(cm, 5, b);
    __syncthreads();
    pmark(C, 5);
}
__device__ ALVRL_POP_INL void commit_ready(CJ& J_in, CC& cm_in, Ctl& C, uint32_t b, uint32_t e)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    if (C.hlds) commit_ready_t<1>(J, cm, C, b, e);
    else commit_ready_t<0>(J, cm, C, b, e);
}

// The leader's split of [b, e): claim a queued task, wait for a running one
// and commit its result, or split here.  While a helper still runs [b, e)
// the leader splits other queued clusters speculatively.  spec = false:
// plain split.
__device__ void split_team(CJ& J_in, CC& cm_in, Ctl& C, uint32_t b, uint32_t e,
                           unsigned long long* lds, Prof& pf, bool spec)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    CT& T = J.team;
    if (!T.helpers || !spec || C.team_off) { heap_move(J, C, false); split(J, cm, C, b, e, lds, pf); return; }
    const int tid = threadIdx.x;
    if (C.hlds && C.heap_n + 2 > kHeapLdsMax) heap_move(J, C, false);   // uniform (after the caller's barrier)
    bool parked = false;   // the heap went back to global memory for a split here
    if (tid < 64 && cm.enq_start) enqueue_candidates(J, cm, C);
    if (tid == 0) {
        publish_tail(T, C);
        trace(cm, 3, b);
        unsigned long long* st = &T.state[b];
        const unsigned long long key = (unsigned long long)e << 3;
        // the word pop_wave fetched: since then it can only have moved on
        // (queued -> running -> done), which the CAS and the wait loop see
        const unsigned long long sv = C.sw;
        int mode = 0;
        if ((uint32_t)(sv >> 3) == e && (sv & 7) == kStDone) {
            mode = 1;   // finished already: commit (sc1 loads of the sc1-stored result, no acquire)
            tcount(cm, TS_COMMIT);
        } else if ((uint32_t)(sv >> 3) == e && (sv & 7) != kStNone && (sv & 7) != kStLeader) {
            if ((sv & 7) == kStQueued && cas_rlx(st, sv, key | kStLeader)) {
                mode = 0;
                tcount(cm, TS_STEAL);
            } else {
                mode = 3;   // running on a helper: wait below, splitting other tasks meanwhile
                C.t0 = wall();
                trace(cm, 4, b);
            }
        } else {
            st_rlx(st, key | kStLeader);
            tcount(cm, TS_OWN);
        }
        C.tmode = mode;
    }
    __syncthreads();
    pf.mark(PF_T_STATE);
#ifndef ALVRL_PT_POP
    pmark(C, 2);
#endif
    while (true) {
        const int tm = C.tmode;
        __syncthreads();   // every thread has read tmode before thread 0 rewrites it
        if (tm != 3) break;
        if (tid == 0) {
            const unsigned long long sv = ld_rlx(&T.state[b]);
            C.side = 0;
            if ((sv & 7) == kStDone && (uint32_t)(sv >> 3) == e) {
                C.tmode = 1;   // the commit reads the result with sc1 loads: no acquire
                tcount(cm, TS_COMMIT);
            } else if (wall() - C.t0 > cm.wait_ticks) {
                // give up on the helper: it still owns team.spec[b, e),
                // team.res[b] and state[b], so the team is retired and the
                // leader splits this and every later cluster of the job itself
                C.tmode = 0;
                C.team_off = 1;
                tcount(cm, TS_WAIT_TMO);
            } else {
                uint32_t yb = 0, ye = 0;
                if (part_try(cm, &yb, &ye)) {   // a part of a divided split (perhaps the awaited one's)
                    C.side = 2; C.yb = yb; C.ye = ye;
                } else {
                    const int got = try_claim(T, &yb, &ye, (uint64_t)(e - b) * cm.side_k / 16);
                    if (got == 1) { C.side = 1; C.yb = yb; C.ye = ye; tcount(cm, TS_LSIDE); }
                    else if (got == 0) __builtin_amdgcn_s_sleep(8);
                }
            }
        }
        __syncthreads();
        pf.mark(PF_T_WAIT);
        if (C.side) {
            if (C.hlds) { heap_move(J, C, false); parked = true; }
            const uint32_t yb = C.yb, ye = C.ye;
            __syncthreads();
            if (C.side == 2) run_part(cm, C, yb, ye, reinterpret_cast<unsigned char*>(lds), false);
            else spec_split(J, view_of(cm, wid_leader(cm, blockIdx.x), blockIdx.x), cm, C, lds, yb, ye);   // (leaders only)
        }
        __syncthreads();
        pf.mark(PF_T_SIDE);
    }
    const int mode = C.tmode;
#ifndef ALVRL_PT_POP
    pmark(C, 3);
#endif
    if (tid == 0 && C.prec) gpw(C.prec)[7] = (uint32_t)mode | (min(e - b, 0xFFFFFFu) << 8);
    if (C.team_off) {   // set by thread 0 before the loop's last barrier
        stop_team(J, cm, C);
        heap_move(J, C, false);
        split(J, cm, C, b, e, lds, pf);
        return;
    }
    if (mode == 0) {
        if (C.hlds) { heap_move(J, C, false); parked = true; }
        split(J, cm, C, b, e, lds, pf);
    }
    if (parked) heap_move(J, C, true);
    if (mode == 1) {
        commit_spec(J, C, b, e);
        pf.mark(PF_T_COMMIT);
    }
#ifndef ALVRL_PT_POP
    pmark(C, 4);
#endif
    // an own split releases its vrls (every wave drained, barrier, one
    // write-back) before its children can be queued; a committed one's
    // children read team.spec
    if (mode == 0) {
        drain_vmem();
        __syncthreads();
    } else if (mode == 1 && tid < 64 && !C.hlds) {
        drain_vmem();   // wave 0 queues from the global heap thread 0 just wrote
    }
    if (tid < 64) {
        if (mode == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        enqueue_candidates(J, cm, C);
    }
    if (tid == 0) trace(cm, 5, b);
    __syncthreads();
    pf.mark(PF_T_ENQ);
    pmark(C, 5);
}

// Setup tasks of a job's first helper (Team::ctl words 4-9, zeroed per
// launch): task 0 = the column weights of [N/2, N), task 1 = the unclustered
// variance.  Either side claims a free task with a CAS (state 0 -> 1); the
// one that ran it publishes the outputs and sets state 2 (producer form of
// spec_split: drained stores, barrier, one agent-scope release, relaxed
// flag).  The leader waits only for a task a running helper has claimed, so
// nothing depends on the helper being resident.  Results are those of the
// leader alone: the same per-column and per-row arithmetic in the same order.
enum : uint32_t { kSuColw = 4, kSuUncl = 5, kSuIntVar = 6, kSuTrVar = 7, kSuUnclErr = 8, kSuColwErr = 9 };
__device__ bool su_claim(CT& T_in, uint32_t task, Ctl& C)
{
    CT& T = uni(T_in);
    if (threadIdx.x == 0) C.go = cas_rlx(&T.ctl[task], 0u, 1u) ? 1 : 0;
    __syncthreads();
    const bool got = C.go != 0;
    __syncthreads();
    return got;
}
__device__ void su_publish(CT& T_in, uint32_t task)
{
    CT& T = uni(T_in);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_rlx(&T.ctl[task], 2u);
    }
    __syncthreads();
}
// the leader's wait for a task a helper has claimed: that helper is running
// and depends on nobody, so the wait ends; it is not bounded by the wait
// knobs (the helper writes colw, which the leader must not finish under it),
// only by a 60 s guard (false: the job fails)
__device__ bool su_wait(CT& T_in, uint32_t task, CC& cm_in, Ctl& C)
{
    CT& T = uni(T_in);
    CC& cm = uni(cm_in);
    if (threadIdx.x == 0) {
        const unsigned long long t0 = wall();
        int ok = 1;
        while (ld_rlx(&T.ctl[task]) != 2u) {
            if (wall() - t0 > kSpinTicks) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(8);
        }
        fence_acq();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        C.go = ok;
    }
    __syncthreads();
    const bool ok = C.go != 0;
    __syncthreads();
    return ok;
}
__device__ void unclustered_variance(CJ& J, CC& cm, Ctl& C, const uint32_t* vrls_in, uint32_t nv);
// the helper's side (Jw: its own scratch, colw shared with the leader)
__device__ void setup_tasks(CJ& J0_in, CJ& Jw_in, CC& cm_in, Ctl& C, bool)
{
    CJ& J0 = uni(J0_in);
    CJ& Jw = uni(Jw_in);
    CC& cm = uni(cm_in);
    CT& T = J0.team;
    const uint32_t N = cm.nvrl;
    // where the leader divides a tall job's column weights (colw_parts) it takes them
    // all: a helper's half on one workgroup would be the setup's critical path
    const bool cparts = cm.parts && cm.proj_min && N >= cm.proj_min &&
                        (J0.nrows > 256 ? cm.part_min_tall : (cm.colw_all ? cm.part_min : 0u));
    if (!cparts && su_claim(T, kSuColw, C)) {
        if (threadIdx.x == 0) C.err = 0;
        __syncthreads();
        EVLOG(cm, 6, N / 2, N);
        colw_raw(Jw, cm, C, N / 2, N);
        EVLOG(cm, 7, N / 2, N);
        if (threadIdx.x == 0) st_rlx(&T.ctl[kSuColwErr], (uint32_t)C.err);
        su_publish(T, kSuColw);
    }
    if (su_claim(T, kSuUncl, C)) {
        if (threadIdx.x == 0) C.err = 0;
        __syncthreads();
        unclustered_variance(Jw, cm, C, cm.init_vrls, cm.init_off[cm.ninit]);
        if (threadIdx.x == 0) {
            st_rlx(&T.ctl[kSuIntVar], __float_as_uint(C.unclIntVar));
            st_rlx(&T.ctl[kSuTrVar], __float_as_uint(C.tracingVar));
            st_rlx(&T.ctl[kSuUnclErr], (uint32_t)C.err);
        }
        su_publish(T, kSuUncl);
    }
    if (threadIdx.x == 0) C.err = 0;
    __syncthreads();
}

// A helper workgroup: split queued clusters of job J until the leader stops.
__device__ __noinline__ void helper_loop(CJ& J0_in, uint32_t j, uint32_t hid, CC& cm_in, Ctl& C,
                                         unsigned long long* lds)
{
    CJ& J0 = uni(J0_in);
    CC& cm = uni(cm_in);
    CT& T = J0.team;
    CJ& J = view_of(cm, wid_helper(cm, j, hid), j);   // vrls = team.spec, this helper's scratch
    const int tid = threadIdx.x;
    if (tid == 0) C.err = 0;
    trace(cm, 10, 0);
    if (hid == 0 && cm.team_setup) setup_tasks(J0, J, cm, C, false);
    while (true) {
        if (tid == 0) {
            const unsigned long long t_idle = wall();
            int got = 0;
            uint32_t b = 0, e = 0;
            if (cm.idle) __hip_atomic_fetch_add(cm.idle, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (true) {
                if (ld_rlx(&T.ctl[2])) { got = -1; break; }
                if (part_try(cm, &b, &e)) { got = 2; break; }   // a part of a divided split first
                const int c = try_claim(T, &b, &e);
                if (c == 1) { got = 1; tcount(cm, TS_HSTART); break; }
                if (c == 2) continue;
                if (wall() - t_idle > cm.spin_ticks) { got = -1; tcount(cm, TS_IDLE_EXIT); break; }
                __builtin_amdgcn_s_sleep(32);
            }
            if (cm.idle) __hip_atomic_fetch_add(cm.idle, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tadd(cm, TS_HIDLE, wall() - t_idle);
            C.go = got; C.b = b; C.e = e;
        }
        __syncthreads();
        if (C.go < 0) break;
        if (C.go == 2) {
            const uint32_t ps = C.b, pp = C.e;
            __syncthreads();
            run_part(cm, C, ps, pp, reinterpret_cast<unsigned char*>(lds), false);
            continue;
        }
        trace(cm, 11, C.b);
        const unsigned long long t_busy = wall();
        spec_split(J0, J, cm, C, lds, C.b, C.e);
        if (tid == 0) { tcount(cm, TS_HDONE); tadd(cm, TS_HBUSY, wall() - t_busy); }
        trace(cm, 12, C.b);
    }
}

// A roaming helper: takes queued clusters from any job's queue (starting
// from the job it last served), splits them with its own scratch.
__device__ __noinline__ void roam_loop(const ALVRL_AS4 JobDev* jobs, uint32_t wid, uint32_t start, CC& cm_in,
                                       Ctl& C, unsigned long long* lds)
{
    CC& cm = uni(cm_in);
    const uint32_t njobs = cm.njobs;
    const int tid = threadIdx.x;
    uint32_t j = start % njobs;
    if (tid == 0) C.err = 0;
    while (true) {
        if (tid == 0) {
            const unsigned long long t_idle = wall();
            int got = 0;
            uint32_t b = 0, e = 0, jj = j;
            if (cm.idle) __hip_atomic_fetch_add(cm.idle, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            while (true) {
                if (part_try(cm, &b, &e)) { got = 2; break; }   // a part of a divided split first
                uint32_t live = 0;
                for (uint32_t k = 0; k < njobs && !got; k++) {
                    jj = cm.roam_order ? cm.roam_order[k] : (j + k < njobs ? j + k : j + k - njobs);
                    CT& T = jobs[jj].team;
                    if (ld_rlx(&T.ctl[2])) continue;
                    live++;
                    int c;
                    do { c = try_claim(T, &b, &e); } while (c == 2);
                    if (c == 1) got = 1;
                }
                if (got) { tcount(cm, TS_HSTART); break; }
                if ((!live && !(cm.parts && ld_rlx(cm.part_open))) || wall() - t_idle > cm.spin_ticks) { got = -1; break; }
                __builtin_amdgcn_s_sleep(32);
            }
            if (cm.idle) __hip_atomic_fetch_add(cm.idle, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tadd(cm, TS_RIDLE, wall() - t_idle);
            C.go = got; C.b = b; C.e = e; C.j = jj;
        }
        __syncthreads();
        if (C.go < 0) break;
        if (C.go == 2) {
            const uint32_t ps = C.b, pp = C.e;
            __syncthreads();
            run_part(cm, C, ps, pp, reinterpret_cast<unsigned char*>(lds), false);
            continue;
        }
        j = C.j;
        CJ& J0 = uni(jobs[j]);
        CJ& Jw = view_of(cm, wid, j);   // vrls = team.spec, this workgroup's scratch
        const unsigned long long t_busy = wall();
        spec_split(J0, Jw, cm, C, lds, C.b, C.e);
        if (tid == 0) { tcount(cm, TS_HDONE); tadd(cm, TS_RBUSY, wall() - t_busy); }
    }
}

// calculateColumnWeigths (:985-1008) with the +1% of the mean (:1002-1007).
// Out of line: inlined into k_refine its loops ran on spilled registers
// (scratch reloads, each a vmcnt(0) wait).
// calculateColumnWeigths' per-column weights of columns [vb, ve) (the part
// a job's helper can take; colw_finish adds the average afterwards)
// (JV: the job, or a part's view of it -- rows, locality weights, colw)
template <class JV>
__device__ __noinline__ void colw_raw(const JV& J_in, CC& cm_in, Ctl& C, uint32_t vb, uint32_t ve)
{
    const JV& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int tid = threadIdx.x, wave = tid >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const uint32_t R = J.nrows;
    // calculateColumnWeigths (:985-1008): one wave per 16 columns, rows in the
    // shared order (lane l sums rows l, l+64, l+128, l+192 from 0, then the halving
    // tree, here transposed: the 16 column sums in one tree16_transposed)
    if (R <= 64u * 4u) {
        const uint32_t NBr = (uint32_t)__builtin_amdgcn_readfirstlane((int)((R + 63) / 64));   // uniform: scalar branches
        const float2* const Rt = cm.Rt;
        auto* const colw = gpw(J.colw);
        constexpr int Q = 16;
        RowRef rr[4];
        double lw[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t r = (uint32_t)b * 64 + lane;
            rr[b] = row_ref(J, min(r, R - 1));
            lw[b] = r < R ? gp(J.locw)[r] : 0.0;
        }
        // the row-block count as a template constant: every load of a group
        // is issued back to back, with no branch between them (a branch per
        // load made the compiler wait for each before issuing the next)
        auto run = [&](auto nbc) {
            constexpr int NB = decltype(nbc)::value;
            for (uint32_t v0 = vb + (uint32_t)wave * Q; v0 < ve; v0 += kWaves * Q) {
                float2 x[NB][Q];
#pragma unroll
                for (int b = 0; b < NB; b++)
#pragma unroll
                    for (int q = 0; q < Q; q++)
                        x[b][q] = ldg2(Rt, rr[b].base + (size_t)min(v0 + (uint32_t)q, ve - 1) * rr[b].stride);
                double v[Q];
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    double p = 0.0;
#pragma unroll
                    for (int b = 0; b < NB; b++) {
                        const double mean = (double)x[b][q].x, var = (double)x[b][q].y;
                        const double xx = mean * mean + var;
                        const double pn = p + lw[b] * xx;
                        p = (uint32_t)b * 64 + lane < R ? pn : p;   // a select, not a branch
                    }
                    v[q] = p;
                }
                const double t = tree16_transposed(v, lane);
                if ((lane & 3) == 0) {
                    const uint32_t j = ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2) | (((lane >> 2) & 1) << 3);
                    if (v0 + j < ve) {
                        const float cw = (float)sqrt(t > 0.0 ? t : 0.0);
                        colw[v0 + j] = cw;
                        if (!isfinite(cw)) C.err = 1;
                    }
                }
            }
        };
        if (NBr <= 1) run(std::integral_constant<int, 1>{});
        else if (NBr == 2) run(std::integral_constant<int, 2>{});
        else if (NBr == 3) run(std::integral_constant<int, 3>{});
        else run(std::integral_constant<int, 4>{});
    } else {
        for (uint32_t v0 = vb + (uint32_t)wave * kCB; v0 < ve; v0 += kWaves * kCB) {
            double p[kCB];
#pragma unroll
            for (int q = 0; q < kCB; q++) p[q] = 0.0;
            for (uint32_t r = lane; r < R; r += 64) {
                const RowRef rr = row_ref(J, r);
                const double lw = J.locw[r];
                float2 mv[kCB];
#pragma unroll
                for (int q = 0; q < kCB; q++) mv[q] = ldg2(cm.Rt, rr.base + (size_t)min(v0 + (uint32_t)q, ve - 1) * rr.stride);
#pragma unroll
                for (int q = 0; q < kCB; q++) {
                    const double mean = (double)mv[q].x, var = (double)mv[q].y;
                    const double x = mean * mean + var;
                    p[q] = p[q] + lw * x;
                }
            }
#pragma unroll
            for (int q = 0; q < kCB; q++) {
                const double t = tree_d(p[q]);
                if (lane == 0 && v0 + q < ve) {
                    const float cw = (float)sqrt(t > 0.0 ? t : 0.0);
                    J.colw[v0 + q] = cw;
                    if (!isfinite(cw)) C.err = 1;
                }
            }
        }
    }
    __syncthreads();
}

// the average of all column weights (running float sum in index order) and
// its 1 % added to every weight (:1002-1007)
__device__ __noinline__ void colw_finish(CJ& J_in, CC& cm_in, Ctl& C)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int tid = threadIdx.x, wave = tid >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const uint32_t N = cm.nvrl;
    if (wave == 0) {
        // the running float sum in index order (one add after the other, as
        // the reference's loop), 64 weights per load, broadcast by v_readlane;
        // 16 loads per lane issued at the top of each step and used within it
        // (a load in flight across the loop's back edge costs a full drain)
        const auto* cwp = gp(J.colw);
        float acc = 0.0f;
        constexpr uint32_t K = 16;
        const uint32_t Nu = (uint32_t)__builtin_amdgcn_readfirstlane((int)N);
        for (uint32_t b0 = 0; b0 < Nu; b0 += K * 64) {
            float x[K];
#pragma unroll
            for (uint32_t k = 0; k < K; k++) x[k] = cwp[min(b0 + k * 64 + lane, Nu - 1)];
#pragma unroll
            for (uint32_t k = 0; k < K; k++) {
                const uint32_t b = b0 + k * 64;
                if (b >= Nu) break;
                if (b + 64 <= Nu) {
#pragma unroll
                    for (int c = 0; c < 64; c++) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[k]), c));
                } else {
                    for (uint32_t c = 0; c < Nu - b; c++) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[k]), c));
                }
            }
        }
        if (lane == 0) {
            float avg = acc / N;
            if (avg == 0) avg = 1.0f;
            C.avg = avg;
        }
    }
    __syncthreads();
    {
        const float add = C.avg * 1e-2f;
        for (uint32_t v = tid; v < N; v += kThreads) J.colw[v] += add;
    }
    __syncthreads();
}

// calculateUnclusteredVariance (:1022-1048), out of line for the same reason
__device__ __noinline__ void unclustered_variance(CJ& J_in, CC& cm_in, Ctl& C, const uint32_t* vrls_in,
                                                  uint32_t nv)
{
    CJ& J = uni(J_in);
    CC& cm = uni(cm_in);
    const int tid = threadIdx.x, wave = tid >> 6;
    const uint32_t lane = (uint32_t)(tid & 63);
    const uint32_t R = J.nrows;
    // calculateUnclusteredVariance (:1022-1048): per-row Welford in m_vrls
    // order, one lane per row; column ids 64 at a time (one per lane, the
    // next block's in flight) broadcast by v_readlane, 1/(n+1) formed once
    // per lane for the block, entries 16 columns ahead
    {
        const uint32_t NBr = (R + 63) / 64;
        const auto* vr = gp(vrls_in);
        constexpr int G = 16;
        for (uint32_t rb = (uint32_t)wave; rb < NBr; rb += kWaves) {
            const uint32_t r = rb * 64 + lane;
            const RowRef rr = row_ref(J, min(r, R - 1));
            const float2* const Rt = cm.Rt + rr.base;
            const size_t rs = rr.stride;
            double mean = 0.0, M2 = 0.0, sv = 0.0;
            uint32_t vid = lane < nv ? vr[lane] : 0u;
            float2 eA[G], eB[G];
            auto load = [&](uint32_t vids, uint32_t g, uint32_t cnt, float2* e) {
#pragma unroll
                for (int k = 0; k < G; k++) {
                    const uint32_t c = g + (uint32_t)k < cnt ? g + (uint32_t)k : 0u;
                    e[k] = ldg2(Rt, (size_t)(uint32_t)__builtin_amdgcn_readlane((int)vids, (int)c) * rs);
                }
            };
            for (uint32_t b = 0; b < nv; b += 64) {
                const uint32_t nvid = b + 64 + lane < nv ? vr[b + 64 + lane] : 0u;
                const uint32_t cnt = min(64u, nv - b);
                const double rnl = 1.0 / (double)(b + lane + 1);
                load(vid, 0, cnt, eA);
                for (uint32_t g = 0; g < cnt; g += G) {
                    if (g + G < cnt) load(vid, g + G, cnt, eB);
#pragma unroll
                    for (int k = 0; k < G; k++) {
                        if (g + (uint32_t)k < cnt) {
                            const double rn = readlane_d(rnl, g + (uint32_t)k);
                            sv = sv + (double)eA[k].y;
                            const double x = (double)eA[k].x;
                            const double delta = x - mean;
                            mean = mean + delta * rn;
                            M2 = M2 + delta * (x - mean);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < G; k++) eA[k] = eB[k];
                }
                vid = nvid;
            }
            if (r < R) { gpw(J.st)[r] = sv; gpw(J.st)[R + r] = M2; }
        }
    }
    __syncthreads();
    if (wave == 0) {
        double pv = 0.0, pm = 0.0;
        for (uint32_t r = lane; r < R; r += 64) {
            pv = pv + J.locw[r] * J.st[r];
            pm = pm + J.locw[r] * J.st[R + r];
        }
        pv = tree_d(pv);
        pm = tree_d(pm);
        if (lane == 0) {
            if (nv <= 1) C.err = 1;
            C.unclIntVar = (float)pv;
            C.tracingVar = (float)(pm - (double)C.unclIntVar);
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------- kernel --
__global__ void __launch_bounds__(kThreads) k_refine(const ALVRL_AS4 JobDev* __restrict__ jobs,
                                                     const ALVRL_AS4 Common* __restrict__ cmp)
{
    CC& cm = *cmp;
    __shared__ Ctl C;
    __shared__ __attribute__((aligned(16))) unsigned char pool[kPoolBytes];
    unsigned long long* lds = reinterpret_cast<unsigned long long*>(pool);
    if (threadIdx.x == 0) {   // one row group; no LDS heap, no trace record until a leader sets them
        C.g_row0 = 0; C.g_first = 1; C.g_last = 1; C.g_carry = nullptr;
        C.hlds = 0; C.hpool = pool; C.prec = nullptr;
    }
    __syncthreads();
    if (blockIdx.x >= cm.njobs * cm.team) {   // a roaming helper
        const uint32_t rid = blockIdx.x - cm.njobs * cm.team;
        roam_loop(jobs, rid, rid * 37u, cm, C, lds);
        trace(cm, 14, 0);
        return;
    }
    if (blockIdx.x >= cm.njobs) {   // a helper of job (blockIdx.x - njobs) / (team - 1)
        const uint32_t h = blockIdx.x - cm.njobs, per = cm.team - 1;
        helper_loop(jobs[h / per], h / per, h % per, cm, C, lds);
        // its job is done: help the others until every job is
        if (cm.roam_on) roam_loop(jobs, wid_helper(cm, h / per, h % per), h / per + 1, cm, C, lds);
        trace(cm, 13, 0);
        return;
    }
    CJ& J = jobs[blockIdx.x];
    trace(cm, 1, 0);
    EVLOG(cm, 1, J.nrows, 0);
    if (cm.jtime && threadIdx.x == 0) cm.jtime[3 * blockIdx.x] = wall();
    const int tid = threadIdx.x, wave = tid >> 6;
    const uint32_t N = cm.nvrl, R = J.nrows;
    const uint32_t nv = cm.init_off[cm.ninit];
    __shared__ Prof pf;
    unsigned long long split_cols = 0;   // thread 0: columns of the clusters split
    if (tid == 0) {
        pf.p = cm.prof; pf.t = (long long)clock64(); pf.sm = -1;
        C.tracingVar = C.unclIntVar = C.clUnderVar = C.clIntVar = 0.0f;
        C.heap_n = C.singles_n = C.sh_heap_n = C.sh_singles_n = 0;
        C.err = 0; C.refined = 1; C.team_off = 0;
        C.hlog_n = 0; C.hlog_full = 1;
        C.prec = nullptr;
        C.hlds = 0; C.hpool = pool;
        C.qpend = 0; C.pre_b = ~0u;
        C.qtail = 0; C.qhead = 0; C.early_b = ~0u;
    }
    __syncthreads();
    const bool tsu = cm.team_setup && cm.team > 1 && J.team.helpers != 0;
    // column ranges on idle workgroups (colw_parts) for wide jobs: the
    // helper's half is claimed first so that nobody computes it twice
    const bool cparts = cm.parts && cm.proj_min && N >= cm.proj_min && (R > 256 ? cm.part_min_tall : cm.part_min);
    if (tsu && cparts && (R > 256 || cm.colw_all) && su_claim(J.team, kSuColw, C)) {
        if (!colw_parts(J, cm, C, 0, N, pool)) colw_raw(J, cm, C, 0, N);
    } else if (tsu) {
        // the first half here, the second on the job's helper unless it
        // has not claimed it yet
        if (!(cparts && colw_parts(J, cm, C, 0, N / 2, pool))) colw_raw(J, cm, C, 0, N / 2);
        if (su_claim(J.team, kSuColw, C)) {
            colw_raw(J, cm, C, N / 2, N);
        } else if (!su_wait(J.team, kSuColw, cm, C)) {
            if (tid == 0) C.err = 1;
        } else if (tid == 0 && ld_rlx(&J.team.ctl[kSuColwErr])) {
            C.err = 1;
        }
        __syncthreads();
    } else if (!(cparts && colw_parts(J, cm, C, 0, N, pool))) {
        colw_raw(J, cm, C, 0, N);
    }
    colw_finish(J, cm, C);
    pf.mark(PF_COLW);
    EVLOG(cm, 2, J.nrows, 0);
    for (uint32_t i = tid; i < nv; i += kThreads) J.vrls[i] = cm.init_vrls[i];
    __syncthreads();
    if (cm.early_spec && cm.team > 1 && J.team.helpers != 0 && J.do_refine && cm.ninit > 0 && !C.err) {
        // the root's split starts on a helper now (its vrls and colw released
        // first: every wave drained, barrier, one agent-scope release)
        drain_vmem();
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            enqueue_early(J, cm, C, cm.init_off[0], cm.init_off[1]);
        }
        __syncthreads();
    }
    // initial clusters
    for (uint32_t i = 0; i < cm.ninit; i += 2) {
        const uint32_t b0 = cm.init_off[i], e0 = cm.init_off[i + 1];
        const bool two = i + 1 < cm.ninit;
        const uint32_t b1 = two ? cm.init_off[i + 1] : 0, e1 = two ? cm.init_off[i + 2] : 0;
        if (b0 == e0 || (two && b1 == e1)) { if (tid == 0) C.err = 1; __syncthreads(); continue; }
        variance_passes(J, cm, C, J.vrls + b0, e0 - b0, 1, nullptr, nullptr, nullptr, nullptr, pool);
        if (tid == 0) add_cluster(J, C, b0, e0, C.vg[0].res_u, C.vg[0].res_i, nullptr, b0 == C.early_b ? kEndQ : 0u);
        __syncthreads();
        if (two) {
            variance_passes(J, cm, C, J.vrls + b1, e1 - b1, 1, nullptr, nullptr, nullptr, nullptr, pool);
            if (tid == 0) add_cluster(J, C, b1, e1, C.vg[0].res_u, C.vg[0].res_i, nullptr, b1 == C.early_b ? kEndQ : 0u);
            __syncthreads();
        }
    }
    pf.mark(PF_INIT);
    EVLOG(cm, 3, J.nrows, 0);
    if (tsu && !su_claim(J.team, kSuUncl, C)) {
        const bool ok = su_wait(J.team, kSuUncl, cm, C);
        if (tid == 0) {
            if (!ok || ld_rlx(&J.team.ctl[kSuUnclErr])) C.err = 1;
            C.unclIntVar = __uint_as_float(ld_rlx(&J.team.ctl[kSuIntVar]));
            C.tracingVar = __uint_as_float(ld_rlx(&J.team.ctl[kSuTrVar]));
        }
        __syncthreads();
    } else {
        unclustered_variance(J, cm, C, cm.init_vrls, nv);
    }
    pf.mark(PF_UNCL);
    EVLOG(cm, 4, J.nrows, 0);
    // release the initial clusters' vrls to the helpers (see split_team)
    drain_vmem();
    __syncthreads();
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();

    // refine (:380-489)
    if (J.do_refine && !C.err) {
        if (J.undersampling > 0) {
            // refineFixedDepth (:387-399)
            const uint32_t target = (uint32_t)(0.5 + (double)((float)N / J.undersampling));
            if (J.team.helpers && cm.heap_lds) heap_move(J, C, true);
            while (true) {
                if (tid < 64) {   // wave 0 decides (every lane reads C itself) and pops (pop_wave)
                    const bool go = (n_clusters(C) < target && C.heap_n > 0 && !C.err);
                    if (tid == 0) C.go = go;
                    if (go) {
                        const CNode cn = pop_wave(J, C, J.team.helpers && !C.team_off ? J.team.state : nullptr);
                        if (tid == 0) { C.b = cn.begin; C.e = cn.end; split_cols += cn.end - cn.begin; }
                    }
                }
                __syncthreads();
                if (!C.go) break;
                if (commit_ready_ok(J, cm, C, C.e)) commit_ready(J, cm, C, C.b, C.e);
                else split_team(J, cm, C, C.b, C.e, lds, pf, true);
            }
            heap_move(J, C, false);
        } else {
            // refineAdaptively (:402-489)
            const float dc = J.depth_correction;
            int run = 0;
            if (tid == 0) {
                if (C.heap_n <= 0) { run = 0; }
                else if (unclustered_var(C) == 0) { C.refined = 0; run = 0; }
                else run = 1;
                C.go = run;
            }
            __syncthreads();
            if (C.go) {
                __shared__ float best;
                __shared__ int nsplit, bestN;
                if (tid == 0) { best = conv_const(C, N, J.pixel_under); nsplit = 0; bestN = 0; }
                snapshot(J, C);
                if (J.team.helpers && cm.heap_lds) heap_move(J, C, true);
                uint32_t npop = 0;
                while (true) {
                    if (tid == 0) {
                        C.prec = cm.poptr && blockIdx.x == cm.poptr_job && npop < cm.poptr_cap ? cm.poptr + 8 * npop : nullptr;
                        npop++;
                    }
                    pmark(C, 0);
                    if (tid < 64) {   // wave 0 decides (every lane reads C itself) and pops (pop_wave)
                        const bool go = C.heap_n > 0 && !C.err;
                        if (tid == 0) C.go = go;
                        if (go) {
                            const CNode cn = pop_wave(J, C, J.team.helpers && !C.team_off ? J.team.state : nullptr);
                            if (tid == 0) { C.b = cn.begin; C.e = cn.end; split_cols += cn.end - cn.begin; }
                        }
                    }
                    __syncthreads();
                    if (!C.go) break;
                    pf.mark(PF_T_HEAP);
#ifdef ALVRL_PT_POP
                    pmark(C, 4);
#else
                    pmark(C, 1);
#endif
                    if (commit_ready_ok(J, cm, C, C.e)) commit_ready(J, cm, C, C.b, C.e);
                    else split_team(J, cm, C, C.b, C.e, lds, pf, true);
                    if (tid == 0) {
                        nsplit++;
                        const float curr = conv_const(C, N, J.pixel_under);
                        C.do_snap = 0;
                        if (curr < best) {
                            if (dc == 1) C.do_snap = 1;
                            best = curr;
                            bestN = nsplit;
                        }
                        C.stop = lower_bound(C, N, J.pixel_under) >= best;
                    }
                    __syncthreads();
                    pf.mark(PF_T_HEAP);
                    if (C.do_snap) snapshot(J, C);
                    pf.mark(PF_T_SNAP);
                    pmark(C, 6);
                    if (C.stop) break;
                }
                if (tid == 0) C.prec = nullptr;
                stop_team(J, cm, C);
                heap_move(J, C, false);
                restore(J, C);
                if (dc != 1) {
                    const int corrected = (int)(0.5 + dc * bestN);
                    for (int i = 0; i < corrected; i++) {
                        if (tid < 64) {   // wave 0 decides (every lane reads C itself) and pops (pop_wave)
                            const bool go = C.heap_n > 0 && !C.err;
                            if (tid == 0) C.go = go;
                            if (go) {
                                const CNode cn = pop_wave(J, C);
                                if (tid == 0) { C.b = cn.begin; C.e = cn.end; split_cols += cn.end - cn.begin; }
                            }
                        }
                        __syncthreads();
                        if (!C.go) break;
                        split_team(J, cm, C, C.b, C.e, lds, pf, false);
                    }
                }
            }
        }
    }
    stop_team(J, cm, C);
    EVLOG(cm, 5, J.nrows, 0);
    if (cm.jtime && threadIdx.x == 0) cm.jtime[3 * blockIdx.x + 1] = wall();
    __syncthreads();
    pf.mark(PF_CTRL);
    // the heap nodes' queue flags off (their ends are the clusters')
    for (int k = tid; k < C.heap_n; k += kThreads) gpw(&J.heap[k].end)[0] = J.heap[k].end & kEndMask;
    __syncthreads();
    // sampleRepresentatives (:354-378)
    // singletons first (std::list push_front order), then one weighted pick
    // per multi-cluster in heap order; every cluster has its own stream, so
    // the picks run one cluster per lane
    const int refined = C.err ? 0 : C.refined;
    const int ns = C.singles_n, nh = C.heap_n;
    __syncthreads();                       // every wave has read C.err before any pick sets it
    if (refined) {
        for (int k = tid; k < ns; k += kThreads) {
            J.out_reps[ns - 1 - k] = J.singles[k];
            J.out_w[ns - 1 - k] = 1.0f;
        }
        for (int k = wave; k < nh; k += kWaves) {   // one wave per multi-cluster
            const CNode cn = J.heap[k];
            Smp smp;
            smp.init(cm.seed, cm.pass, cn.begin, cn.end, J.stage_sample);
            const WsPick pk = weighted_sample_wave(nullptr, J.colw, J.vrls + cn.begin, cn.end - cn.begin, smp,
                                                   0xFFFFFFFFu, true);
            if ((threadIdx.x & 63) == 0) {
                if (pk.err) atomicOr(&C.err, 1);
                J.out_reps[ns + k] = J.vrls[cn.begin + pk.idx];
                J.out_w[ns + k] = 1.0f / pk.prob;
            }
        }
    }
    __syncthreads();
    if (J.out_members) {
        // getVrlsPerCluster (:526-543): singletons in list order (newest
        // first), then the heap's clusters in its vector order
        for (int k = tid; k < ns; k += kThreads) {
            J.out_members[k] = J.singles[ns - 1 - k];
            J.out_moff[k + 1] = (uint32_t)(k + 1);
        }
        if (tid == 0) {
            J.out_moff[0] = 0;
            uint32_t at = (uint32_t)ns;
            for (int k = 0; k < nh; k++) { at += J.heap[k].end - J.heap[k].begin; J.out_moff[ns + k + 1] = at; }
            *J.out_nclusters = (uint32_t)(ns + nh);
        }
        __syncthreads();
        for (int k = 0; k < nh; k++) {
            const CNode cn = J.heap[k];
            const uint32_t at = J.out_moff[ns + k];
            for (uint32_t j = cn.begin + (uint32_t)tid; j < cn.end; j += kThreads) J.out_members[at + (j - cn.begin)] = J.vrls[j];
        }
    }
    __syncthreads();
    pf.mark(PF_REPS);
    if (tid == 0) {
        *J.out_n = refined ? (uint32_t)(ns + nh) : 0u;
        *J.out_refined = refined;
        *J.out_err = C.err;
        // column weights, initial clusters and unclustered variance read every
        // entry once; a split reads its cluster's columns (at least) once
        if (cm.entries) {
            gadd(&cm.entries[0], (3ull * N + split_cols) * R);
            gadd(&cm.entries[1], split_cols * R);
        }
    }
    if (cm.jtime && tid == 0) cm.jtime[3 * blockIdx.x + 2] = wall();
    if (cm.roam_on) {
        // this job is done: its leader helps the others with its own scratch
        __syncthreads();
        roam_loop(jobs, wid_leader(cm, blockIdx.x), blockIdx.x + 1, cm, C, lds);
    }
}

// Packs the jobs' representative lists back to back (job order) so the host
// fetches every result with three copies: meta[3j..3j+2] = (n, refined, err).
// Common::views: job j with vrls = team.spec and workgroup w's split scratch
// (a roamer's, a helper's or a leader's own), one view per thread
__global__ void __launch_bounds__(256) k_views(const JobDev* __restrict__ jobs, const Common* __restrict__ cmp,
                                               JobDev* __restrict__ views)
{
    const Common& cm = *cmp;
    const uint32_t nj = cm.njobs, G = cm.team, nh = nj * (G - 1);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (cm.nroam + nh + nj) * nj) return;
    const uint32_t w = i / nj, j = i % nj;
    JobDev v = jobs[j];
    v.vrls = jobs[j].team.spec;
    SplitWs ws;
    if (w < cm.nroam) {
        ws = cm.roam_ws[w];
    } else if (w < cm.nroam + nh) {
        const uint32_t h = w - cm.nroam;
        ws = jobs[h / (G - 1)].team.ws[h % (G - 1)];
    } else {
        const JobDev& o = jobs[w - cm.nroam - nh];
        ws = SplitWs{o.dir, o.st, o.bufM, o.keys0, o.keys1, o.fsu, o.fsi, o.feu, o.fei, o.carry};
    }
    v.dir = ws.dir; v.st = ws.st; v.bufM = ws.bufM; v.keys0 = ws.keys0; v.keys1 = ws.keys1;
    v.fsu = ws.fsu; v.fsi = ws.fsi; v.feu = ws.feu; v.fei = ws.fei; v.carry = ws.carry;
    views[i] = v;
}

__global__ void __launch_bounds__(256) k_pack_results(const JobDev* __restrict__ jobs, uint32_t njobs,
                                                      uint32_t nvrl, uint32_t* __restrict__ meta,
                                                      uint32_t* __restrict__ reps, float* __restrict__ w)
{
    const uint32_t j = blockIdx.x;
    __shared__ unsigned long long off;
    if (threadIdx.x == 0) {
        unsigned long long o = 0;
        for (uint32_t i = 0; i < j; i++) o += min(*jobs[i].out_n, nvrl);
        off = o;
    }
    __syncthreads();
    const JobDev& J = jobs[j];
    const uint32_t n = min(*J.out_n, nvrl);
    for (uint32_t k = threadIdx.x; k < n; k += 256) {
        reps[off + k] = J.out_reps[k];
        w[off + k] = J.out_w[k];
    }
    if (threadIdx.x == 0) {
        meta[3 * j] = *J.out_n;
        meta[3 * j + 1] = (uint32_t)*J.out_refined;
        meta[3 * j + 2] = (uint32_t)*J.out_err;
    }
}

// ------------------------------------------------------------- host --
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct HostJob {
    const uint32_t* rows;
    const double* locw;
    uint32_t nrows;
    float pixel_under, undersampling, depth_correction;
    int do_refine;
    uint32_t stage_refine, stage_sample;
    const uint64_t* row_off;      // optional per-row layout, see alvrl_cluster_job
    const uint32_t* row_stride;
    uint32_t* members;            // optional getVrlsPerCluster outputs (host): ids,
    uint32_t* moff;               //   offsets (clusters + 1) and the cluster count
    uint32_t* nclusters;
};

// Runs every clustering job on the device (one workgroup each) and copies the
// representatives back.  Returns 0 or an ALVRL_ERR_* code with *err set.
// Device scratch of refine_jobs kept by the caller between calls (grow-only):
// a ~1 GB hipMalloc / hipFree pair per prepass costs milliseconds of host time
// on the critical path (hipFree also waits for the device).
void RefineArenas::release()
{
    if (arena) (void)hipFree(arena);
    if (tarena) (void)hipFree(tarena);
    if (varena) (void)hipFree(varena);
    arena = tarena = varena = nullptr;
    arena_cap = tarena_cap = varena_cap = 0;
}
static hipError_t arena_get(char** buf, size_t* cap, size_t bytes, bool cached)
{
    if (cached && *buf && *cap >= bytes) return hipSuccess;
    if (*buf) { (void)hipFree(*buf); *buf = nullptr; *cap = 0; }
    const size_t want = cached ? bytes + bytes / 4 : bytes;   // slack for the next pass's sizes
    hipError_t e = hipMalloc(buf, want);
    if (e != hipSuccess && want != bytes) { (void)hipGetLastError(); e = hipMalloc(buf, bytes); if (e == hipSuccess) *cap = bytes; }
    else if (e == hipSuccess) *cap = want;
    if (e != hipSuccess) *buf = nullptr;
    return e;
}

int refine_jobs(hipStream_t s, const float* d_Rt, uint64_t ld, uint32_t nvrl, uint32_t seed,
                uint32_t pass, uint32_t njobs, const HostJob* jobs, const uint32_t* init_vrls,
                const uint32_t* init_off, uint32_t ninit, uint32_t* out_off, uint32_t* out_reps,
                float* out_w, int* out_refined, float* ms, unsigned long long* entries, std::string* err,
                RefineArenas* cache)
{
    RefineArenas local;
    RefineArenas& ar = cache ? *cache : local;
    struct Finally {
        RefineArenas* l;
        ~Finally() { if (l) l->release(); }
    } fin{cache ? nullptr : &local};
    if (ms) *ms = 0.0f;
    if (entries) entries[0] = entries[1] = 0;
    out_off[0] = 0;
    if (njobs == 0) return 0;
    // the initial clusters partition the VRLs they list (every VRL for the
    // per-slice jobs; the non-zero ones for clusterRefinement, :899-912)
    const uint32_t nv = init_off[ninit];
    if (nv > nvrl) { *err = "alvrl_refine: initial clusters list more VRLs than there are"; return 1; }
    for (uint32_t i = 0; i < ninit; i++)
        if (init_off[i + 1] < init_off[i]) { *err = "alvrl_refine: init_off not monotone"; return 1; }
    {
        std::vector<unsigned char> seen(nvrl, 0);
        for (uint32_t i = 0; i < nv; i++) {
            if (init_vrls[i] >= nvrl || seen[init_vrls[i]]) { *err = "alvrl_refine: initial clusters are not disjoint"; return 1; }
            seen[init_vrls[i]] = 1;
        }
    }
    const size_t N = nvrl;
    std::vector<size_t> row_off(njobs), job_off(njobs);
    size_t rows_total = 0;
    for (uint32_t j = 0; j < njobs; j++) {
        if (jobs[j].nrows == 0) { *err = "alvrl_refine: job with no rows"; return 1; }
        row_off[j] = rows_total;
        rows_total += jobs[j].nrows;
    }
    // Team size from the occupancy: teams of G workgroups for njobs jobs are
    // resident together when njobs * G <= resident blocks; the rest of the
    // resident capacity gets roaming helpers.  ALVRL_REFINE_TEAM=n caps G
    // (1 = no speculation).
    const char* bs_env = std::getenv("ALVRL_REFINE_BATCH");
    uint32_t G = 1, nroam = 0;
    {
        int ncu = 0, nb = 0, dev = 0;
        const char* te = std::getenv("ALVRL_REFINE_TEAM");
        const uint32_t cap = te ? (uint32_t)std::max(1, std::atoi(te)) : 8u;
        if (!bs_env && hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_refine, kThreads, 0) == hipSuccess && nb > 0)
            G = std::min<uint32_t>(cap, (uint32_t)(nb * ncu) / njobs);
        if (G < 2) G = 1;
        // the CUs the teams leave free get roaming helpers (ALVRL_REFINE_ROAM=0: none)
        const char* re = std::getenv("ALVRL_REFINE_ROAM");
        if (cap > 1 && nb > 0 && (!re || std::atoi(re) != 0) && (uint32_t)(nb * ncu) > njobs * G)
            nroam = std::min<uint32_t>((uint32_t)(nb * ncu) - njobs * G, 1024u);
        // ALVRL_REFINE_NROAM=n: at most n roaming helpers of their own (the CUs
        // left to other work launched beside the refinement)
        if (const char* nr = std::getenv("ALVRL_REFINE_NROAM")) nroam = std::min<uint32_t>(nroam, (uint32_t)std::max(0, std::atoi(nr)));
    }
    const bool team_on = G > 1 || nroam > 0;
    // finished leaders and helpers roam too: their split scratch is sized for
    // the largest job
    const bool roam_on = team_on && !(std::getenv("ALVRL_REFINE_ROAM") && std::atoi(std::getenv("ALVRL_REFINE_ROAM")) == 0);
    uint32_t Rmax = 0;
    for (uint32_t j = 0; j < njobs; j++) Rmax = std::max(Rmax, jobs[j].nrows);
    auto job_bytes = [&](const HostJob& H) {
        const uint32_t R = roam_on ? Rmax : H.nrows;
        return align_up(N * 4) * 2 + align_up(N * sizeof(CNode)) * 2 + align_up(N * 4) * 2 +
               align_up((size_t)R * 4) + align_up(N * 8) * 2 + align_up(N * 4) * 4 +
               align_up((size_t)6 * R * 8) + align_up((size_t)2 * 2 * kCH * ((R + 63) / 64) * 64 * 16) +
               align_up(N * 4) * 2 + align_up(16) + (H.members ? align_up(N * 4) + align_up((N + 1) * 4) + align_up(4) : 0) +
               (R > 256 ? align_up((size_t)4 * N * 8) : 0);
    };
    size_t total = align_up(rows_total * 8) + align_up(rows_total * 4) + align_up(rows_total * 8) + align_up((size_t)nv * 4) +
                   align_up((size_t)(ninit + 1) * 4) + align_up((size_t)njobs * sizeof(JobDev)) +
                   align_up((size_t)njobs * 12) + 2 * align_up((size_t)njobs * N * 4) + align_up(16);
    for (uint32_t j = 0; j < njobs; j++) { job_off[j] = total; total += job_bytes(jobs[j]); }
    hipError_t e = arena_get(&ar.arena, &ar.arena_cap, total, cache != nullptr);
    if (e != hipSuccess) { *err = std::string("alvrl_refine: hipMalloc: ") + hipGetErrorString(e); return 4; }
    char* const arena = ar.arena;
    size_t o = 0;
    unsigned long long* d_roff = (unsigned long long*)(arena + o); o += align_up(rows_total * 8);
    uint32_t* d_rstride = (uint32_t*)(arena + o); o += align_up(rows_total * 4);
    double* d_locw = (double*)(arena + o); o += align_up(rows_total * 8);
    uint32_t* d_init = (uint32_t*)(arena + o); o += align_up((size_t)nv * 4);
    uint32_t* d_init_off = (uint32_t*)(arena + o); o += align_up((size_t)(ninit + 1) * 4);
    JobDev* d_jobs = (JobDev*)(arena + o); o += align_up((size_t)njobs * sizeof(JobDev));
    uint32_t* d_meta = (uint32_t*)(arena + o); o += align_up((size_t)njobs * 12);
    uint32_t* d_preps = (uint32_t*)(arena + o); o += align_up((size_t)njobs * N * 4);
    float* d_pw = (float*)(arena + o); o += align_up((size_t)njobs * N * 4);
    unsigned long long* d_entries = (unsigned long long*)(arena + o);
    std::vector<unsigned long long> h_roff(rows_total);
    std::vector<uint32_t> h_rstride(rows_total);
    std::vector<double> h_locw(rows_total);
    std::vector<JobDev> h_jobs(njobs);
    for (uint32_t j = 0; j < njobs; j++) {
        const HostJob& H = jobs[j];
        for (uint32_t r = 0; r < H.nrows; r++) {
            if (H.row_off) {
                if (H.row_stride[r] == 0) { *err = "alvrl_refine: zero row stride"; return 1; }
                h_roff[row_off[j] + r] = H.row_off[r];
                h_rstride[row_off[j] + r] = H.row_stride[r];
            } else {
                if (H.rows[r] >= ld) { *err = "alvrl_refine: row id out of range"; return 1; }
                if (ld > 0xFFFFFFFFull) { *err = "alvrl_refine: ld too large"; return 1; }
                h_roff[row_off[j] + r] = H.rows[r];
                h_rstride[row_off[j] + r] = (uint32_t)ld;
            }
            h_locw[row_off[j] + r] = H.locw[r];
        }
        JobDev& J = h_jobs[j];
        char* p = arena + job_off[j];
        const uint32_t R = H.nrows, Rw = roam_on ? Rmax : R;
        J.roff = d_roff + row_off[j]; J.rstride = d_rstride + row_off[j];
        J.locw = d_locw + row_off[j]; J.nrows = R;
        const unsigned long long* ho = &h_roff[row_off[j]];
        const uint32_t* hs = &h_rstride[row_off[j]];
        J.off0 = ho[0]; J.stride0 = hs[0];
        J.contig = 1;
        for (uint32_t r = 0; r < R; r++)
            if (ho[r] != ho[0] + r || hs[r] != hs[0]) { J.contig = 0; break; }
        J.pixel_under = H.pixel_under; J.undersampling = H.undersampling;
        J.depth_correction = H.depth_correction; J.do_refine = H.do_refine;
        J.stage_refine = H.stage_refine; J.stage_sample = H.stage_sample;
        J.vrls = (uint32_t*)p; p += align_up(N * 4);
        J.colw = (float*)p; p += align_up(N * 4);
        J.heap = (CNode*)p; p += align_up(N * sizeof(CNode));
        J.sh_heap = (CNode*)p; p += align_up(N * sizeof(CNode));
        J.singles = (uint32_t*)p; p += align_up(N * 4);
        J.sh_singles = (uint32_t*)p; p += align_up(N * 4);
        J.dir = (float*)p; p += align_up((size_t)Rw * 4);
        J.keys0 = (unsigned long long*)p; p += align_up(N * 8);
        J.keys1 = (unsigned long long*)p; p += align_up(N * 8);
        J.fsu = (float*)p; p += align_up(N * 4);
        J.fsi = (float*)p; p += align_up(N * 4);
        J.feu = (float*)p; p += align_up(N * 4);
        J.fei = (float*)p; p += align_up(N * 4);
        J.carry = nullptr;
        if (Rw > 256) { J.carry = (double*)p; p += align_up((size_t)4 * N * 8); }
        J.st = (double*)p; p += align_up((size_t)6 * Rw * 8);
        J.bufM = (double*)p; p += align_up((size_t)2 * 2 * kCH * ((Rw + 63) / 64) * 64 * 16);   // T, 2 passes x 2 chunks
        J.bufV = nullptr;
        J.out_reps = (uint32_t*)p; p += align_up(N * 4);
        J.out_w = (float*)p; p += align_up(N * 4);
        J.out_n = (uint32_t*)p;
        J.out_refined = (int*)(p + 4);
        J.out_err = (int*)(p + 8);
        p += align_up(16);
        J.out_members = J.out_moff = J.out_nclusters = nullptr;
        if (H.members) {
            J.out_members = (uint32_t*)p; p += align_up(N * 4);
            J.out_moff = (uint32_t*)p; p += align_up((N + 1) * 4);
            J.out_nclusters = (uint32_t*)p;
        }
    }
    char* tarena = nullptr;
    size_t tbytes = 0, board_off = 0, board_ctl = 0, slot_T = 0, slot_Ts = 0, board_T = 0;
    uint32_t nslots = 0, nbig = 0, nsmall = 0, small_cap = 0, part_min = 0, part_min_tall = 0, part_blk = 4;
    bool busy_launch = false;
    if (team_on) {
        auto helper_bytes = [&](uint32_t R) {
            return align_up((size_t)R * 4) + align_up((size_t)6 * R * 8) +
                   align_up((size_t)2 * 2 * kCH * ((R + 63) / 64) * 64 * 16) + 2 * align_up(N * 8) + 4 * align_up(N * 4) +
                   (R > 256 ? align_up((size_t)4 * N * 8) : 0);
        };
        const size_t team_fixed = align_up(N * 4) + align_up(N * 8) + align_up(N * sizeof(SplitRes)) +
                                  align_up((size_t)kQueue * 8) + align_up(16) + align_up((size_t)(G - 1) * sizeof(SplitWs));
        for (uint32_t j = 0; j < njobs; j++) tbytes += team_fixed + (size_t)(G - 1) * helper_bytes(roam_on ? Rmax : jobs[j].nrows);
        tbytes += align_up((size_t)nroam * sizeof(SplitWs)) + (size_t)nroam * helper_bytes(Rmax);
        tbytes += align_up((size_t)njobs * 4);   // roam order
        // the part board after everything else: slots, the open count, and
        // each slot's block totals (4 x 64-row blocks x N doubles; only the
        // control words are cleared per launch)
        board_off = tbytes;
        // (a busy launch gates the short jobs' parts on many idle workgroups, below)
        const char* pm = std::getenv("ALVRL_PART_MIN");
        part_min = pm ? (uint32_t)std::max(0, std::atoi(pm)) : 4096u;
        busy_launch = njobs * 3u > njobs * G + nroam;
        const char* pt = std::getenv("ALVRL_PART_MIN_TALL");
        part_min_tall = pt ? (uint32_t)std::max(0, std::atoi(pt)) : (pm ? std::min(part_min, 257u) : 257u);
        const char* pb = std::getenv("ALVRL_PART_BLK");
        part_blk = pb ? (uint32_t)std::min(std::max(1, std::atoi(pb)), (int)kPartMaxBlk) : 4u;
        if (part_min || (part_min_tall && Rmax > 256)) {
            // big slots (any split, up to N columns) within ALVRL_PART_MB (default
            // 16 GB, at most a quarter of the free memory), small ones (up to
            // ALVRL_PART_SMALL columns) for the many mid-size splits of tall jobs
            const char* ps = std::getenv("ALVRL_PART_SLOTS");
            const char* pmb = std::getenv("ALVRL_PART_MB");
            const char* psc = std::getenv("ALVRL_PART_SMALL");
            const size_t nbk = (Rmax + 63) / 64;
            slot_T = align_up((size_t)4 * nbk * N * 8);
            small_cap = std::min<uint32_t>(psc ? (uint32_t)std::max(0, std::atoi(psc)) : 16384u, (uint32_t)N);
            slot_Ts = align_up((size_t)4 * nbk * std::max<uint32_t>(small_cap, 1u) * 8);
            size_t budget = (pmb ? (size_t)std::max(1, std::atoi(pmb)) : 16384u) << 20;
            size_t fr = 0, tot = 0;
            if (!pmb && hipMemGetInfo(&fr, &tot) == hipSuccess) budget = std::min(budget, fr / 4);
            const uint32_t wgs = njobs * G + nroam;
            nbig = (uint32_t)std::min<size_t>(ps ? (size_t)std::max(0, std::atoi(ps)) : 64u, budget / slot_T);
            nbig = std::min<uint32_t>(nbig, wgs);
            nsmall = small_cap < N ? std::min<uint32_t>(wgs, (uint32_t)std::min<size_t>(256u, (budget / 8) / slot_Ts)) : 0u;
            nslots = nbig + nsmall;
        }
        board_ctl = nslots ? align_up((size_t)nslots * sizeof(PartSlot)) + align_up(8) : 0;
        board_T = nbig * slot_T + nsmall * slot_Ts;
        if (arena_get(&ar.tarena, &ar.tarena_cap, tbytes + board_ctl + board_T, cache != nullptr) != hipSuccess) {
            (void)hipGetLastError();
            nslots = nbig = nsmall = 0; board_ctl = board_T = 0;   // without the board
            if (arena_get(&ar.tarena, &ar.tarena_cap, tbytes, cache != nullptr) != hipSuccess) {
                (void)hipGetLastError(); G = 1; nroam = 0;
            }
        }
        tarena = ar.tarena;
    }
    std::vector<SplitWs> h_ws(G > 1 ? (size_t)njobs * (G - 1) : 0), h_rws(nroam);
    SplitWs* d_rws = nullptr;
    {
        size_t to = 0;
        for (uint32_t j = 0; j < njobs; j++) {
            Team& T = h_jobs[j].team;
            T = Team{0u, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
            if (!tarena) continue;
            const uint32_t R = roam_on ? Rmax : jobs[j].nrows;
            char* q = tarena + to;
            T.helpers = (G - 1) + (nroam + njobs - 1) / njobs;
            T.spec = (uint32_t*)q; q += align_up(N * 4);
            T.state = (unsigned long long*)q; q += align_up(N * 8);
            T.res = (SplitRes*)q; q += align_up(N * sizeof(SplitRes));
            T.queue = (unsigned long long*)q; q += align_up((size_t)kQueue * 8);
            T.ctl = (uint32_t*)q; q += align_up(16);
            T.ws = (const SplitWs*)q; q += align_up((size_t)(G - 1) * sizeof(SplitWs));
            for (uint32_t h = 0; h + 1 < G; h++) {
                SplitWs& w = h_ws[(size_t)j * (G - 1) + h];
                w.dir = (float*)q; q += align_up((size_t)R * 4);
                w.st = (double*)q; q += align_up((size_t)6 * R * 8);
                w.bufM = (double*)q; q += align_up((size_t)2 * 2 * kCH * ((R + 63) / 64) * 64 * 16);
                w.keys0 = (unsigned long long*)q; q += align_up(N * 8);
                w.keys1 = (unsigned long long*)q; q += align_up(N * 8);
                w.fsu = (float*)q; q += align_up(N * 4);
                w.fsi = (float*)q; q += align_up(N * 4);
                w.feu = (float*)q; q += align_up(N * 4);
                w.fei = (float*)q; q += align_up(N * 4);
                w.carry = nullptr;
                if (R > 256) { w.carry = (double*)q; q += align_up((size_t)4 * N * 8); }
            }
            to = (size_t)(q - tarena);
        }
        if (tarena && nroam) {
            auto carve = [&](size_t n) { char* q = tarena + to; to += align_up(n); return q; };
            d_rws = (SplitWs*)carve((size_t)nroam * sizeof(SplitWs));
            for (uint32_t r = 0; r < nroam; r++) {
                SplitWs& w = h_rws[r];
                w.dir = (float*)carve((size_t)Rmax * 4);
                w.st = (double*)carve((size_t)6 * Rmax * 8);
                w.bufM = (double*)carve((size_t)2 * 2 * kCH * ((Rmax + 63) / 64) * 64 * 16);
                w.keys0 = (unsigned long long*)carve(N * 8);
                w.keys1 = (unsigned long long*)carve(N * 8);
                w.fsu = (float*)carve(N * 4);
                w.fsi = (float*)carve(N * 4);
                w.feu = (float*)carve(N * 4);
                w.fei = (float*)carve(N * 4);
                w.carry = Rmax > 256 ? (double*)carve((size_t)4 * N * 8) : nullptr;
            }
        }
    }
    Common cm;
    cm.Rt = reinterpret_cast<const float2*>(d_Rt); cm.ld = ld; cm.nvrl = nvrl;
    cm.njobs = njobs; cm.team = G;
    cm.nroam = nroam; cm.roam_ws = d_rws;
    cm.roam_on = roam_on && tarena ? 1 : 0;
    {
        // ALVRL_FINISHED_ROAM=0: finished leaders and helpers exit instead of roaming
        const char* fr = std::getenv("ALVRL_FINISHED_ROAM");
        if (fr && fr[0] == '0') cm.roam_on = 0;
    }
    {
        const char* sw = std::getenv("ALVRL_SPEC_WIDTH");
        // C4 refine sweeps: round 1 (tools/env_sweep.sh, min 2) width 24 401 ms, 32 398; round 5,
        // after the fused small split (tools/env_sweep2.sh, tools/w8_width.sh, profiles/r05/sweep/):
        // N = 1 (a busy launch) 32 260.4, 56 257.1, 128 258.1-258.4, 192 259.9-260.8, 256 262.3-262.8
        // ms; C4 rank 0 of 8 32 127-133, 56 115-122, 128 106-109, 192 104-107 ms
        cm.spec_width = sw ? (uint32_t)std::max(1, std::atoi(sw)) : (busy_launch ? 128u : 192u);
    }
    {
        const char* sp = std::getenv("ALVRL_REFINE_SPIN_MS");
        cm.spin_ticks = sp ? (unsigned long long)std::max(1, std::atoi(sp)) * 100000ull : kSpinTicks;
        // ALVRL_LEADER_WAIT_TICKS (test knob, may be 0): bound of a leader's
        // wait for a running helper; by default the same as an idle helper's
        const char* wt = std::getenv("ALVRL_LEADER_WAIT_TICKS");
        cm.wait_ticks = wt ? std::strtoull(wt, nullptr, 10) : cm.spin_ticks;
        // ALVRL_SORT_RADIX_MIN (developer knob, 0: never): the split sort's radix threshold.
        // C4 refine (profiles/r05/sort/): 16,385 243.7 ms, 4,096 241.8, 1,024 240.0; bitonic only 258
        const char* rm = std::getenv("ALVRL_SORT_RADIX_MIN");
        const long rmv = rm ? std::atol(rm) : 1024L;
        cm.sort_radix_min = rmv <= 0 ? 0xFFFFFFFFu : (uint32_t)std::min<long>(std::max<long>(rmv, 2L), 0x7FFFFFFFL);
        // ALVRL_WS_WG_MIN (developer knob, 0: never): the split's weighted picks on every wave
        const char* wm = std::getenv("ALVRL_WS_WG_MIN");
        const long wmv = wm ? std::atol(wm) : 4096L;
        cm.ws_wg_min = wmv <= 0 ? 0xFFFFFFFFu : (uint32_t)std::min<long>(std::max<long>(wmv, 2L), 0x7FFFFFFFL);
    }
    cm.tstat = nullptr;
    cm.trace = nullptr;
    const char* tre = std::getenv("ALVRL_REFINE_TRACE");
    if (tre && tre[0] == '1' && hipHostMalloc(&cm.trace, 256 * 8, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess)
        std::memset(cm.trace, 0, 256 * 8);
    else
        cm.trace = nullptr;
    const char* tse = std::getenv("ALVRL_REFINE_TEAM_STATS");
    cm.jtime = nullptr;
    if (team_on && tse && tse[0] == '1' && hipMalloc(&cm.tstat, TS_N * 8) == hipSuccess) {
        (void)hipMemsetAsync(cm.tstat, 0, TS_N * 8, s);
        if (hipMalloc(&cm.jtime, (size_t)njobs * 3 * 8) != hipSuccess) cm.jtime = nullptr;
    }
    {
        const char* sm = std::getenv("ALVRL_SPEC_MIN");
        cm.spec_min = sm ? (uint32_t)std::max(2, std::atoi(sm)) : 2u;   // width 16: min 32 447 ms, 16 422, 8 413, 4 409, 2 407
        const char* sk = std::getenv("ALVRL_LEADER_SIDE");
        cm.side_k = sk ? (uint32_t)std::max(0, std::atoi(sk)) : 1u << 24;
        const char* es = std::getenv("ALVRL_ENQ_START");
        cm.enq_start = es ? std::atoi(es) : 0;   // queueing after the commit only: 398 vs 401 ms at width 32
        const char* tsu = std::getenv("ALVRL_TEAM_SETUP");
        cm.team_setup = tsu ? std::atoi(tsu) : 1;
        const char* esp = std::getenv("ALVRL_EARLY_SPEC");
        cm.early_spec = esp ? std::atoi(esp) : 1;
        const char* hl = std::getenv("ALVRL_HEAP_LDS");
        cm.heap_lds = hl ? std::atoi(hl) : 1;
    }
    // ALVRL_ROAM_ORDER=1: roaming helpers scan the jobs with the most rows
    // first.  Measured slower (C4 refine 436 vs 420 ms: the roamers crowd the
    // big jobs' short queues and the leaders claim more of their own work), so
    // by default each roamer rotates from the job it served last.
    std::vector<uint32_t> h_order;
    cm.roam_order = nullptr;
    {
        const char* ro = std::getenv("ALVRL_ROAM_ORDER");
        if (tarena && cm.roam_on && ro && ro[0] == '1') {
            h_order.resize(njobs);
            for (uint32_t j = 0; j < njobs; j++) h_order[j] = j;
            std::stable_sort(h_order.begin(), h_order.end(),
                             [&](uint32_t a, uint32_t b) { return jobs[a].nrows > jobs[b].nrows; });
            cm.roam_order = (const uint32_t*)(tarena + board_off - align_up((size_t)njobs * 4));
        }
    }
    cm.parts = nullptr; cm.nslots = 0; cm.part_min = part_min; cm.part_blk = part_blk; cm.part_open = nullptr;
    cm.nbig = 0; cm.small_cap = 0; cm.idle = nullptr;
    {
        const char* pbs = std::getenv("ALVRL_PART_BLK_SHORT");
        cm.part_blk_short = pbs ? (uint32_t)std::min(std::max(1, std::atoi(pbs)), (int)kPartMaxBlk) : 2u;
        const char* pbi = std::getenv("ALVRL_PART_BLK_INIT");
        cm.part_blk_init = pbi ? (uint32_t)std::min(std::max(1, std::atoi(pbi)), (int)kPartMaxBlk) : 1u;
    }
    {
        const char* im = std::getenv("ALVRL_PART_IDLE");
        cm.idle_min = im ? (uint32_t)std::max(0, std::atoi(im)) : 1u;
        // jobs of <= 256 rows in a busy launch (about a third as many jobs as
        // resident workgroups or more): divided only when many workgroups
        // idle, as in the launch's tail -- the one-workgroup engines do more
        // per CU (C4 at N = 1: 305 against 312-320 ms with parts throughout)
        const char* ims = std::getenv("ALVRL_PART_IDLE_SHORT");
        cm.idle_min_short = ims ? (uint32_t)std::max(0, std::atoi(ims)) : (busy_launch ? 16u : cm.idle_min);
        const char* pr = std::getenv("ALVRL_PART_RED");
        cm.part_red = !(pr && pr[0] == '0');
        const char* ca = std::getenv("ALVRL_COLW_ALL");
        cm.colw_all = ca ? (ca[0] == '1') : !busy_launch;
    }
    cm.part_min_tall = part_min_tall;
    {
        const char* pm = std::getenv("ALVRL_PROJ_MIN");
        cm.proj_min = pm ? (uint32_t)std::max(0, std::atoi(pm)) : 16384u;
        const char* pc = std::getenv("ALVRL_PROJ_CPP");
        cm.proj_cpp = pc ? (uint32_t)std::max(64, std::atoi(pc)) : 16384u;
    }
    std::vector<PartSlot> h_slots;
    if (tarena && nslots) {
        cm.parts = (PartSlot*)(tarena + board_off);
        cm.part_open = (uint32_t*)(tarena + board_off + align_up((size_t)nslots * sizeof(PartSlot)));
        cm.idle = cm.part_open + 1;
        cm.nslots = nslots; cm.nbig = nbig; cm.small_cap = small_cap;
        h_slots.assign(nslots, PartSlot{});
        for (uint32_t k = 0; k < nslots; k++)
            h_slots[k].T = (double*)(tarena + board_off + board_ctl +
                                     (k < nbig ? k * slot_T : nbig * slot_T + (k - nbig) * slot_Ts));
    }
    cm.init_vrls = d_init; cm.init_off = d_init_off; cm.ninit = ninit;
    cm.seed = seed; cm.pass = pass;
    cm.prof = nullptr;
    cm.entries = d_entries;
    {
        const char* vv = std::getenv("ALVRL_VAR_V3");
        cm.var_v3 = !(vv && vv[0] == '0');
        const char* vs = std::getenv("ALVRL_VAR_SMALL");
        cm.var_small = !(vs && vs[0] == '0');
        const char* sf = std::getenv("ALVRL_SPLIT_FUSED");
        cm.split_fused = sf ? std::min(std::max(std::atoi(sf), 0), 2) : 2;
    }
    const char* pe = std::getenv("ALVRL_REFINE_PROFILE");
    if (pe && pe[0] == '1' && hipMalloc(&cm.prof, kPfTotal * 8) == hipSuccess)
        (void)hipMemsetAsync(cm.prof, 0, kPfTotal * 8, s);
    // ALVRL_POP_TRACE=1: the leader of the job with the most rows records the
    // wall clock at 7 points of each pop (tools: the summary printed below)
    cm.poptr = nullptr; cm.poptr_job = 0; cm.poptr_cap = 0;
    // ALVRL_EVLOG=file: the developer event log of a -DALVRL_EVLOG build, written to file
    cm.evlog = nullptr; cm.evlog_n = nullptr; cm.evlog_cap = 0;
    const char* evf = std::getenv("ALVRL_EVLOG");
    if (evf && evf[0]) {
        cm.evlog_cap = 1u << 20;
        if (hipMalloc(&cm.evlog, (size_t)cm.evlog_cap * 24 + 256) == hipSuccess) {
            cm.evlog_n = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(cm.evlog) + (size_t)cm.evlog_cap * 24);
            (void)hipMemsetAsync(cm.evlog_n, 0, 4, s);
        } else {
            cm.evlog = nullptr; cm.evlog_cap = 0;
        }
    }
    {
        const char* pt = std::getenv("ALVRL_POP_TRACE");
        if (pt && pt[0] == '1') {
            uint32_t jm = 0;
            for (uint32_t j = 1; j < njobs; j++) if (jobs[j].nrows > jobs[jm].nrows) jm = j;
            cm.poptr_job = jm; cm.poptr_cap = 32768;
            if (hipMalloc(&cm.poptr, (size_t)cm.poptr_cap * 32) == hipSuccess)
                (void)hipMemsetAsync(cm.poptr, 0, (size_t)cm.poptr_cap * 32, s);
            else
                cm.poptr = nullptr;
        }
    }
    // the kernel's Common and, with helpers or roamers, every workgroup's view
    // of every job (k_views), in device memory read through the constant
    // address space
    const size_t nviews = team_on && tarena ? (size_t)(nroam + njobs * G) * njobs : 0;
    e = arena_get(&ar.varena, &ar.varena_cap, align_up(sizeof(Common)) + nviews * sizeof(JobDev), cache != nullptr);
    if (e != hipSuccess) { *err = std::string("alvrl_refine: hipMalloc: ") + hipGetErrorString(e); return 4; }
    Common* const d_cm = reinterpret_cast<Common*>(ar.varena);
    JobDev* const d_views = nviews ? reinterpret_cast<JobDev*>(ar.varena + align_up(sizeof(Common))) : nullptr;
    cm.views = (const ALVRL_AS4 JobDev*)(uintptr_t)d_views;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipMemcpyAsync(d_roff, h_roff.data(), rows_total * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_rstride, h_rstride.data(), rows_total * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_locw, h_locw.data(), rows_total * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_init, init_vrls, (size_t)nv * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_init_off, init_off, (size_t)(ninit + 1) * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_jobs, h_jobs.data(), njobs * sizeof(JobDev), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemsetAsync(d_entries, 0, 16, s);
    if (e == hipSuccess && tarena) e = hipMemsetAsync(tarena, 0, board_off + board_ctl, s);
    if (e == hipSuccess && cm.parts)
        e = hipMemcpyAsync(cm.parts, h_slots.data(), (size_t)nslots * sizeof(PartSlot), hipMemcpyHostToDevice, s);
    for (uint32_t j = 0; j < njobs && e == hipSuccess && G > 1; j++)
        e = hipMemcpyAsync(const_cast<SplitWs*>(h_jobs[j].team.ws), &h_ws[(size_t)j * (G - 1)],
                           (size_t)(G - 1) * sizeof(SplitWs), hipMemcpyHostToDevice, s);
    if (e == hipSuccess && nroam)
        e = hipMemcpyAsync(d_rws, h_rws.data(), (size_t)nroam * sizeof(SplitWs), hipMemcpyHostToDevice, s);
    if (e == hipSuccess && cm.roam_order)
        e = hipMemcpyAsync(const_cast<uint32_t*>(cm.roam_order), h_order.data(), (size_t)njobs * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_cm, &cm, sizeof(Common), hipMemcpyHostToDevice, s);
    if (e == hipSuccess && nviews) {
        hipLaunchKernelGGL(k_views, dim3((uint32_t)((nviews + 255) / 256)), dim3(256), 0, s, d_jobs, d_cm, d_views);
        e = hipGetLastError();
    }
    const auto* const a_jobs = (const ALVRL_AS4 JobDev*)(uintptr_t)d_jobs;
    const auto* const a_cm = (const ALVRL_AS4 Common*)(uintptr_t)d_cm;
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    if (e == hipSuccess && team_on && tarena) {
        // sized to the resident capacity, but correct without co-residency:
        // no workgroup ever waits for one that has not started (a leader waits
        // only on a cluster a running helper has claimed, helpers only poll),
        // so a late helper finds its job stopped and leaves
        hipLaunchKernelGGL(k_refine, dim3(njobs * G + nroam), dim3(kThreads), 0, s, a_jobs, a_cm);
        e = hipGetLastError();
    } else if (e == hipSuccess) {
        // ALVRL_REFINE_BATCH=n (developer knob): launch the jobs n at a time,
        // to separate per-CU cost from contention between concurrent jobs
        const char* bs = bs_env;
        const uint32_t batch = bs ? (uint32_t)std::max(1, std::atoi(bs)) : njobs;
        for (uint32_t j0 = 0; j0 < njobs && e == hipSuccess; j0 += batch) {
            hipLaunchKernelGGL(k_refine, dim3(std::min(batch, njobs - j0)), dim3(kThreads), 0, s, a_jobs + j0, a_cm);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (cm.trace && e == hipSuccess) {
        // print every block's (phase, value) whenever it changes, until the kernel ends
        const uint32_t nblk = std::min<uint32_t>(256, njobs * G + nroam);
        std::vector<unsigned long long> last(nblk, ~0ull);
        const auto t0 = std::chrono::steady_clock::now();
        while (hipEventQuery(e1) == hipErrorNotReady) {
            std::string line;
            for (uint32_t b = 0; b < nblk; b++) {
                const unsigned long long v = __atomic_load_n(&cm.trace[b], __ATOMIC_RELAXED);
                if (v != last[b]) {
                    last[b] = v;
                    line += " b" + std::to_string(b) + "=" + std::to_string(v >> 32) + ":" + std::to_string((uint32_t)v);
                }
            }
            if (!line.empty())
                std::fprintf(stderr, "[trace %.2f s]%s\n",
                             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), line.c_str());
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
        }
    }
#ifdef ALVRL_LDS_CHECK
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    unsigned int viol = 0;
    if (e == hipSuccess) e = hipMemcpyFromSymbol(&viol, HIP_SYMBOL(g_lds_viol), sizeof(viol));
    if (e == hipSuccess && viol) {
        const unsigned int zero = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lds_viol), &zero, sizeof(zero));
        std::fprintf(stderr, "[refine] ALVRL_LDS_CHECK: %u LDS-pool bounds violations\n", viol);
        *err = "alvrl_refine: LDS-pool bounds violation (ALVRL_LDS_CHECK)";
        return 1;
    }
#endif
    // gather results: packed on the device, three copies
    std::vector<uint32_t> meta(3 * (size_t)njobs);
    unsigned long long h_entries[2] = {0, 0};
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_pack_results, dim3(njobs), dim3(256), 0, s, d_jobs, njobs, nvrl, d_meta, d_preps, d_pw);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(meta.data(), d_meta, (size_t)njobs * 12, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(h_entries, d_entries, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (entries) { entries[0] = h_entries[0]; entries[1] = h_entries[1]; }
    unsigned long long jt_start_traced = 0;   // the pop-traced job's start (wall ticks), with team stats
    if (cm.tstat) {
        unsigned long long h[TS_N];
        if (hipMemcpy(h, cm.tstat, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
            std::fprintf(stderr, "[refine team] G=%u roam=%u jobs=%u enqueued %llu helper start %llu done %llu | leader "
                         "commit %llu steal %llu wait-timeout %llu own %llu side %llu | helper idle exits %llu\n",
                         G, nroam, njobs, h[TS_ENQ], h[TS_HSTART], h[TS_HDONE], h[TS_COMMIT], h[TS_STEAL],
                         h[TS_WAIT_TMO], h[TS_OWN], h[TS_LSIDE], h[TS_IDLE_EXIT]);
            std::fprintf(stderr, "[refine team] wall ms summed: team helpers idle %.0f busy %.0f | roamers (incl. "
                         "finished helpers) idle %.0f busy %.0f\n", h[TS_HIDLE] * 1e-5, h[TS_HBUSY] * 1e-5,
                         h[TS_RIDLE] * 1e-5, h[TS_RBUSY] * 1e-5);
            std::fprintf(stderr, "[refine team] speculative splits' hand-offs, wall ms summed: acquire %.1f, release %.1f "
                         "(%.2f / %.2f us each)\n", h[TS_ACQ] * 1e-5, h[TS_REL] * 1e-5,
                         h[TS_HSTART] ? h[TS_ACQ] * 1e-2 / h[TS_HSTART] : 0.0, h[TS_HSTART] ? h[TS_REL] * 1e-2 / h[TS_HSTART] : 0.0);
            std::fprintf(stderr, "[refine team] split parts: %u slots (%u for any split, %u up to %u columns), min %u / %u "
                         "(> 256 rows) columns, %u blocks per part | divided "
                         "splits %llu (no free slot %llu), parts by owner %llu, by others %llu, owner wait ms summed %.1f\n",
                         cm.nslots, cm.nbig, cm.nslots - cm.nbig, cm.small_cap, cm.part_min, cm.part_min_tall, cm.part_blk,
                         h[TS_PSPLIT], h[TS_PSOLO], h[TS_POWN], h[TS_POTHER],
                         h[TS_PWAIT] * 1e-5);
        }
        hipFree(cm.tstat);
        if (cm.jtime) {
            std::vector<unsigned long long> jt((size_t)njobs * 3);
            if (hipMemcpy(jt.data(), cm.jtime, jt.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                unsigned long long t0 = ~0ull;
                for (uint32_t j = 0; j < njobs; j++) t0 = std::min(t0, jt[3 * j]);
                std::vector<double> fin(njobs), dur(njobs);
                for (uint32_t j = 0; j < njobs; j++) {
                    fin[j] = (jt[3 * j + 2] - t0) * 1e-5;          // ms (100 MHz ticks)
                    dur[j] = (jt[3 * j + 1] - jt[3 * j]) * 1e-5;
                }
                std::vector<double> f2 = fin;
                std::sort(f2.begin(), f2.end());
                const uint32_t jmax = (uint32_t)(std::max_element(fin.begin(), fin.end()) - fin.begin());
                std::fprintf(stderr, "[refine team] job end ms: min %.1f p10 %.1f median %.1f p90 %.1f max %.1f "
                             "(job %u, %u rows, refine %.1f ms)\n", f2.front(), f2[njobs / 10], f2[njobs / 2],
                             f2[(njobs * 9) / 10], f2.back(), jmax, jobs[jmax].nrows, dur[jmax]);
                if (cm.poptr) jt_start_traced = jt[3 * cm.poptr_job];
            }
            hipFree(cm.jtime);
        }
    }
    if (cm.evlog) {
        uint32_t n = 0;
        if (hipMemcpy(&n, cm.evlog_n, 4, hipMemcpyDeviceToHost) == hipSuccess) {
            n = std::min(n, cm.evlog_cap);
            std::vector<unsigned long long> ev((size_t)n * 3);
            FILE* f = n && hipMemcpy(ev.data(), cm.evlog, ev.size() * 8, hipMemcpyDeviceToHost) == hipSuccess
                          ? std::fopen(evf, "a") : nullptr;
            if (f) {
                std::fprintf(f, "# launch: %u jobs, %u events\n", njobs, n);
                for (uint32_t i = 0; i < n; i++)
                    std::fprintf(f, "%llu %u %u %u %u\n", ev[3 * i], (uint32_t)(ev[3 * i + 1] >> 32), (uint32_t)ev[3 * i + 1],
                                 (uint32_t)(ev[3 * i + 2] >> 32), (uint32_t)ev[3 * i + 2]);
                std::fclose(f);
            }
        }
        hipFree(cm.evlog);
    }
    if (cm.poptr) {
        std::vector<uint32_t> pr((size_t)cm.poptr_cap * 8);
        if (hipMemcpy(pr.data(), cm.poptr, pr.size() * 4, hipMemcpyDeviceToHost) == hipSuccess) {
            // segments (100 MHz ticks -> us): pop, state, wait loop, commit or own split,
            // release + queueing, convergence test + snapshot, back to the next pop
            const char* nm[7] = {"pop", "state check", "wait loop", "commit/own split", "queueing", "conv+snapshot", "loop"};
            std::vector<double> seg[7], segc[7];
            uint32_t n = 0, nc = 0;
            for (uint32_t p = 0; p < cm.poptr_cap; p++) {
                const uint32_t* r = &pr[(size_t)p * 8];
                if (r[0] == 0 || r[6] == 0) break;
                const bool quick = (r[7] & 255u) == 1 && (r[3] - r[2]) < 500;   // committed, waited < 5 us
                for (int k = 0; k < 7; k++) {
                    const uint32_t a = r[k], b = k < 6 ? r[k + 1] : (p + 1 < cm.poptr_cap ? pr[(size_t)(p + 1) * 8] : 0u);
                    if (k == 6 && b == 0) continue;
                    seg[k].push_back((b - a) * 1e-2);
                    if (quick) segc[k].push_back((b - a) * 1e-2);
                }
                n++; nc += quick;
            }
            auto stat = [](std::vector<double> v, double* mean, double* p50, double* p90) {
                if (v.empty()) { *mean = *p50 = *p90 = 0; return; }
                double t = 0; for (double x : v) t += x;
                std::sort(v.begin(), v.end());
                *mean = t / v.size(); *p50 = v[v.size() / 2]; *p90 = v[v.size() * 9 / 10];
            };
            std::fprintf(stderr, "[pop trace] job %u (%u rows): %u pops, %u committed without a wait; us per pop "
                         "(all: mean p50 p90 | committed w/o wait: mean p50)\n", cm.poptr_job, jobs[cm.poptr_job].nrows, n, nc);
            double tot = 0, totc = 0;
            for (int k = 0; k < 7; k++) {
                double m, a, b, mc, ac, bc;
                stat(seg[k], &m, &a, &b); stat(segc[k], &mc, &ac, &bc);
                tot += m * seg[k].size(); totc += mc;
                std::fprintf(stderr, "  %-18s %8.2f %8.2f %8.2f | %8.2f %8.2f\n", nm[k], m, a, b, mc, ac);
            }
            std::fprintf(stderr, "  total %.1f ms over the pops; a committed pop without a wait %.2f us\n", tot * 1e-3, totc);
            if (jt_start_traced && n)
                std::fprintf(stderr, "  first pop %.1f ms after the job's start (column weights, initial clusters, "
                             "unclustered variance)\n", (uint32_t)(pr[0] - (uint32_t)jt_start_traced) * 1e-5);
            // waits (wait loop > 5 us) by log2 of the popped cluster's size, and when they happen
            double wt[32] = {0}; uint32_t wn[32] = {0};
            for (uint32_t p = 0; p < n; p++) {
                const uint32_t* r = &pr[(size_t)p * 8];
                const double w = (r[3] - r[2]) * 1e-2;
                if (w < 5.0) continue;
                const uint32_t m = r[7] >> 8;
                const int lb = m ? 31 - __builtin_clz(m) : 0;
                wt[lb] += w; wn[lb]++;
            }
            for (int lb = 0; lb < 32; lb++)
                if (wn[lb]) std::fprintf(stderr, "  waits on clusters of %7u-%7u columns: %5u, %8.2f ms, %8.1f us each\n",
                                         1u << lb, (2u << lb) - 1, wn[lb], wt[lb] * 1e-3, wt[lb] / wn[lb]);
            const uint32_t t0 = pr[0];
            for (int q = 1; q <= 4; q++) {   // pops done by each quarter of the traced time
                const uint32_t lim = t0 + (uint32_t)((double)(pr[(size_t)(n - 1) * 8 + 6] - t0) * q / 4);
                uint32_t c = 0;
                while (c < n && pr[(size_t)c * 8 + 6] <= lim) c++;
                std::fprintf(stderr, "  pops finished by %d/4 of the time: %u\n", q, c);
            }
        }
        hipFree(cm.poptr);
    }
    if (cm.prof) {
        unsigned long long h[kPfTotal];
        if (hipMemcpy(h, cm.prof, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess) {
            unsigned long long tot = 0;
            for (int i = 0; i < PF_NSPLIT; i++) tot += h[i];
            std::fprintf(stderr, "[refine profile] %u jobs, lane-0 cycles summed over jobs:\n", njobs);
            for (int i = 0; i < PF_N; i++)
                std::fprintf(stderr, "  %-22s %16llu%s\n", kPfNames[i], h[i],
                             i < PF_NSPLIT ? (std::string("  ") + std::to_string(100.0 * h[i] / (tot ? tot : 1)).substr(0, 5) + "%").c_str() : "");
            for (int c = 0; c < 2; c++)
                for (int w = 0; w < kWaves; w++) {
                    const unsigned long long* hb = h + kPfWaveBusy + 3 * kWaves * c;
                    const double wall = (double)(hb[kWaves + w] ? hb[kWaves + w] : 1);
                    std::fprintf(stderr, "  variance wave %d (clusters >= 4096 columns, %s rows): step busy %llu (%.1f%%), "
                                 "reduce busy %llu (%.1f%%) of %llu cycles\n", w, c ? "193-256" : "<= 192",
                                 hb[w], 100.0 * hb[w] / wall, hb[2 * kWaves + w], 100.0 * hb[2 * kWaves + w] / wall, hb[kWaves + w]);
                }
            for (int c = 0; c < kPfSmall; c++) {
                unsigned long long n = 0;
                for (int b = 0; b < kPfBuckets; b++)
                    if (c == 0 ? (1u << b) < 64u : ((1u << b) >= 64u && (1u << b) < 256u)) n += h[PF_N + 4 * b];
                std::fprintf(stderr, "  splits of %s columns, cycles per split:", c ? "64-255" : "< 64");
                for (int i = 0; i < kPfSmallPh; i++)
                    std::fprintf(stderr, " %s %.0f", kPfNames[PF_WSAMP + i] + 7, (double)h[kPfSmallAt + c * kPfSmallPh + i] / (n ? n : 1));
                std::fprintf(stderr, "\n");
            }
            std::fprintf(stderr, "  split columns   #splits   cycles/split   variance/split   pre-proj/split   cycles/column   %%cycles\n");
            unsigned long long stot = 0;
            for (int b = 0; b < kPfBuckets; b++) stot += h[PF_N + 4 * b + 1];
            for (int b = 0; b < kPfBuckets; b++) {
                const unsigned long long n = h[PF_N + 4 * b];
                if (!n) continue;
                const double cs = (double)h[PF_N + 4 * b + 1] / n;
                std::fprintf(stderr, "  [%6u,%6u) %9llu %14.0f %16.0f %16.0f %15.1f %8.2f\n", 1u << b, 2u << b, n, cs,
                             (double)h[PF_N + 4 * b + 2] / n, (double)h[PF_N + 4 * b + 3] / n, cs / (1.5 * (1u << b)),
                             100.0 * h[PF_N + 4 * b + 1] / (stot ? stot : 1));
            }
        }
        hipFree(cm.prof);
    }
    int rc = 0;
    if (e == hipSuccess) {
        uint32_t off = 0;
        for (uint32_t j = 0; j < njobs; j++) {
            const uint32_t n = meta[3 * (size_t)j];
            const int refined = (int)meta[3 * (size_t)j + 1];
            const int jerr = (int)meta[3 * (size_t)j + 2];
#ifndef ALVRL_EXP_NOCHAIN   // timing variants with invalid results do not report them
            if (jerr) { rc = 5; *err = "alvrl_refine: clustering invariant violated in job " + std::to_string(j); }
#else
            (void)jerr;
#endif
            if (n > nvrl) { rc = 5; *err = "alvrl_refine: corrupt representative count"; break; }
            out_refined[j] = refined;
            off += n;
            out_off[j + 1] = off;
        }
        if (off) {
            e = hipMemcpyAsync(out_reps, d_preps, (size_t)off * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipMemcpyAsync(out_w, d_pw, (size_t)off * 4, hipMemcpyDeviceToHost, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        for (uint32_t j = 0; j < njobs && e == hipSuccess; j++) {
            if (!jobs[j].members) continue;
            uint32_t nc = 0;
            e = hipMemcpy(&nc, h_jobs[j].out_nclusters, 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) break;
            if (nc > nv) { rc = 5; *err = "alvrl_refine: corrupt cluster count"; break; }
            *jobs[j].nclusters = nc;
            e = hipMemcpy(jobs[j].moff, h_jobs[j].out_moff, (size_t)(nc + 1) * 4, hipMemcpyDeviceToHost);
            if (e == hipSuccess && nv) e = hipMemcpy(jobs[j].members, h_jobs[j].out_members, (size_t)nv * 4, hipMemcpyDeviceToHost);
        }
        if (e == hipSuccess && ms) e = hipEventElapsedTime(ms, e0, e1);
    }
    if (e != hipSuccess) { rc = 3; *err = std::string("alvrl_refine: ") + hipGetErrorString(e); }

    if (cm.trace) hipHostFree(cm.trace);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    return rc;
}

}  // namespace alvrl
