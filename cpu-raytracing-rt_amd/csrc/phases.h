// phases.h — diagnostics of the path kernel (tools/phases.py); compiled in only
// with -DRT_PHASES, so product builds carry none of it.
#pragma once
#include <hip/hip_runtime.h>

namespace rt {

// ---- diagnostics: wave cycles per code region (tools/phases.py) ----------
// Only in -DRT_PHASES builds: s_memtime deltas, added once per wave by the
// first active lane into LDS, flushed to raw stats words 16..16 + kPhN - 1 (16..51).
// The last four words count BVH traversal-loop iterations (wave-level and
// summed over lanes) and primitive tests (wave-level inner-loop trips and
// lane-level tests): their ratios are the loop's SIMD utilisation.  Wave
// cycles inside the resumable walk's steps (trav_step): kPhLeafCyc the steps
// that test leaf primitives, kPhInnerCyc the inner-node visits, kPhPopCyc the
// stack pops, kPhStepCyc whole steps (kPhTris minus it: the loop around them).
// Regions timed with PH_ADDW also add cycles x (active lanes / 64) at k + kPhW:
// the ratio of the two is the region's lane utilisation.  kPhInnerUni counts the
// compact inner-node wave steps whose lanes all visit the same node.  kPhIdleWin /
// kPhIdleDrain count, per path-loop trip, the lanes left without a path after the
// hand-out: held by the commit window (or the open wave-tile cap) while the queue
// still has work, vs the queue drained (the launch tail).
enum { kPhAssign, kPhIntersect, kPhLightSample, kPhLightPdf, kPhSegment, kPhCommit, kPhTile,
       kPhTravWave, kPhTravLane, kPhLeafWave, kPhLeafLane, kPhRngWave, kPhRngLane, kPhW0,
       kPhPlanes = kPhW0 + 5, kPhBoxes, kPhElls, kPhTris, kPhMaterialise,
       kPhInnerWave, kPhInnerLane, kPhLiveLane, kPhIdleWin, kPhIdleDrain,
       kPhPushLane, kPhPushGlobal, kPhPopGlobal, kPhLeafCyc, kPhInnerCyc, kPhPopCyc, kPhStepCyc, kPhInnerUni, kPhN };  // traversal-stack pushes, past the LDS part
static_assert(16 + kPhN <= 52, "phase words fit the raw stats below the timeline words (render.h kTimeline)");
constexpr int kPhW = kPhW0 - kPhIntersect;  // weighted word of region k = k + kPhW (k in 1..5)
#ifdef RT_PHASES
__shared__ unsigned long long g_phase[kPhN];
#define PH_T() __builtin_amdgcn_s_memtime()
#define PH_FIRST() (__lane_id() == (unsigned)__builtin_amdgcn_readfirstlane(__lane_id()))
// (atomics, so the compiler cannot keep a lane-private copy across iterations)
#define PH_ADD(k, t0)                                                                        \
    do {                                                                                     \
        const unsigned long long dt_ = PH_T() - (t0);                                        \
        if (PH_FIRST()) atomicAdd(&g_phase[k], dt_);                                         \
    } while (0)
#define PH_COUNT(kw, kl)                                                                     \
    do {                                                                                     \
        if (PH_FIRST()) atomicAdd(&g_phase[kw], 1ull);                                       \
        atomicAdd(&g_phase[kl], 1ull);                                                       \
    } while (0)
#define PH_LANE(kl) atomicAdd(&g_phase[kl], 1ull)
#define PH_ADDW(k, t0)                                                                       \
    do {                                                                                     \
        const unsigned long long dt_ = PH_T() - (t0);                                        \
        const unsigned long long act_ = (unsigned long long)__popcll(__ballot(1));           \
        if (PH_FIRST()) {                                                                    \
            atomicAdd(&g_phase[k], dt_);                                                     \
            atomicAdd(&g_phase[(k) + kPhW], dt_ * act_ / 64ull);                             \
        }                                                                                    \
    } while (0)
#else
#define PH_T() 0ull
#define PH_ADD(k, t0) ((void)(t0))
#define PH_ADDW(k, t0) ((void)(t0))
#define PH_COUNT(kw, kl) ((void)0)
#define PH_LANE(kl) ((void)0)
#endif

}  // namespace rt
