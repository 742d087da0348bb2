// pekf_run_multi.hip -- the multi-record instantiations of the fused stream kernel (pekf_step.hpp):
// the headline launch of main_file.py:38-47 over a whole resident window (config 3: 10,000 records
// per launch).  A file of its own because it is compiled with the max-ILP machine scheduler
// (Makefile RUNMULTIFLAGS): the time loop's record is ~300 dependent FP64 VALU instructions with
// seven transcendental seeds, and at its 3-4 waves per SIMD (1 at config 2) the interleaving the
// scheduler finds is worth more than the occupancy-first default (same box: config 3 -0.9 %,
// config 2 -4.5 %, profiles/r2/ab_sched_maxilp/).  The one-record and per-record kernels, which move
// state through HBM and want occupancy, stay in pekf_run.hip with the default scheduler.
// Scheduling moves instructions, never their arithmetic: the two files' variants round identically.
#include "pekf_step.hpp"

namespace pekf {

// The PIN schedule of ekf_record_step (the Schur inverse in the Wahba chain's basic block) for the
// FP64 multi-record launch without trajectories or counts: config 2 (one wave per SIMD, the record's
// dependency chain exposed) -2.3 %, config 3 unchanged within noise in an order-balanced A/B
// (profiles/r2/ab_pin_schur/).  PEKF_RUN_PIN=0 selects the compiler's default order (A/B runs, tests).
static bool pin_schedule() {
    const char *e = getenv("PEKF_RUN_PIN");
    return !(e && e[0] == '0');
}

// The HOIST schedule (ekf_record_step) for launches of at most one wave per SIMD (batch <= CUs x 4 x 64:
// config 2's 65,536 filters on 256 CUs), where the record's dependency chain is exposed; more waves fill
// the stalls themselves and pay for the longer block's registers (profiles/r5/ab_hoist/).
// PEKF_RUN_HOIST=0 / 1 forces it off / on (A/B runs, tests).
static bool hoist_schedule(int64_t batch) {
    const char *e = getenv("PEKF_RUN_HOIST");
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return false;
    return batch <= (int64_t)cus * 4 * kWave;
}

int launch_run_multi(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const float4 *gd,
                     const float4 *am, const float2 *my, const double *dtx, const double *refs, double *X,
                     double *P, double q, double r, double *traj, const int32_t *counts, bool mixed, bool soa,
                     hipStream_t stream) {
    const dim3 grid(grid_for(batch, kRunBlock)), block(kRunBlock);
    if (!traj && !mixed && !counts && !dtx && pin_schedule()) {
        if (hoist_schedule(batch)) {
            if (soa)
                hipLaunchKernelGGL((k_run<false, false, true, false, false, true, false, true>), grid, block, 0, stream,
                                   batch, n_steps, window, step0, gd, am, my, refs, X, P, q, r, traj, counts, dtx);
            else
                hipLaunchKernelGGL((k_run<false, false, false, false, false, true, false, true>), grid, block, 0, stream,
                                   batch, n_steps, window, step0, gd, am, my, refs, X, P, q, r, traj, counts, dtx);
        } else if (soa)
            hipLaunchKernelGGL((k_run<false, false, true, false, false, true>), grid, block, 0, stream, batch, n_steps,
                               window, step0, gd, am, my, refs, X, P, q, r, traj, counts, dtx);
        else
            hipLaunchKernelGGL((k_run<false, false, false, false, false, true>), grid, block, 0, stream, batch, n_steps,
                               window, step0, gd, am, my, refs, X, P, q, r, traj, counts, dtx);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_run");
        return PEKF_OK;
    }
#define PEKF_LAUNCH_RUN(TR, MX, SO, CN, LD)                                                                    \
    hipLaunchKernelGGL((k_run<TR, MX, SO, CN, false, false, LD>), grid, block, 0, stream, batch, n_steps, window, \
                       step0, gd, am, my, refs, X, P, q, r, traj, counts, dtx)
#define PEKF_LAUNCH_RUN0(TR, MX, SO, CN) \
    do { if (dtx) PEKF_LAUNCH_RUN(TR, MX, SO, CN, true); else PEKF_LAUNCH_RUN(TR, MX, SO, CN, false); } while (0)
#define PEKF_LAUNCH_RUN1(TR, MX, SO) \
    do { if (counts) PEKF_LAUNCH_RUN0(TR, MX, SO, true); else PEKF_LAUNCH_RUN0(TR, MX, SO, false); } while (0)
#define PEKF_LAUNCH_RUN2(TR, MX) \
    do { if (soa) PEKF_LAUNCH_RUN1(TR, MX, true); else PEKF_LAUNCH_RUN1(TR, MX, false); } while (0)
    if (traj) {
        if (mixed) PEKF_LAUNCH_RUN2(true, true); else PEKF_LAUNCH_RUN2(true, false);
    } else {
        if (mixed) PEKF_LAUNCH_RUN2(false, true); else PEKF_LAUNCH_RUN2(false, false);
    }
#undef PEKF_LAUNCH_RUN2
#undef PEKF_LAUNCH_RUN1
#undef PEKF_LAUNCH_RUN0
#undef PEKF_LAUNCH_RUN
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_run");
    return PEKF_OK;
}

}  // namespace pekf
