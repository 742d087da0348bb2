// pekf_tile.hpp -- coalesced access to per-item (AoS) operands for the per-call kernels.
//
// The per-call API takes NumPy-shaped arrays: item i's W doubles are contiguous (P is
// (n, 4, 4), gyro (n, 3) ...).  Read directly, lane i of a wave touches item i's W doubles, so a
// wave instruction lands on 64 different lines W * 8 bytes apart and the kernel runs at the
// address-processing rate, not at HBM rate (k_correct: 0.16 of HBM peak).  Instead each wave
// moves its 64 items as one contiguous block of 64 * W doubles -- consecutive lanes on
// consecutive doubles, 512 B per wave instruction -- and transposes it through a private slice
// of LDS:
//
//   gather<W>     global -> registers, coalesced (c[j] = block[lane + 64 j])
//   to_lanes<W>   registers -> LDS -> registers, lane l ends up with item l's W doubles
//   from_lanes<W> the reverse, before scatter<W> writes the block back coalesced
//
// LDS layout: item l's doubles at l * S + k with S = W rounded up to odd, so that the per-lane
// reads and writes (ds_*_b64, 32- or 16-lane groups) hit distinct banks; the block-order side
// then sits at e + e / W for even W (shift + add: W is 4 or 16) and at e for odd W.
// Only one wave touches a slice and LDS instructions of a wave execute in order, so no barrier
// is needed: a wavefront-scope fence keeps the compiler from reordering the LDS accesses.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pekf {

constexpr int kWave = 64;

template <int W>
constexpr int tile_stride() {
    return W % 2 ? W : W + 1;
}

// doubles of LDS one wave needs for operands of up to W doubles per item
template <int W>
constexpr int tile_doubles() {
    return kWave * tile_stride<W>();
}

struct WaveTile {
    double *lds;     // this wave's slice
    int64_t first;   // first item of the wave
    int nvalid;      // items of the wave that exist (the last wave of a launch may be short)
    int lane;

    __device__ __forceinline__ WaveTile(double *pool, int slice_doubles, int64_t n) {
        const int wave = threadIdx.x / kWave;
        lane = threadIdx.x % kWave;
        lds = pool + wave * slice_doubles;
        first = ((int64_t)blockIdx.x * blockDim.x) + wave * kWave;
        const int64_t left = n - first;
        nvalid = left >= kWave ? kWave : (left > 0 ? (int)left : 0);
    }

    __device__ __forceinline__ bool active() const { return lane < nvalid; }

    __device__ __forceinline__ static void order() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

    // LDS slot of block element lane + 64 j (j unrolled: a constant offset from one base when W
    // divides 64, so the compiler keeps one address register instead of W)
    template <int W>
    __device__ __forceinline__ int slot(int j) const {
        if constexpr (W % 2) {
            return lane + kWave * j;
        } else if constexpr (kWave % W == 0) {
            return lane + lane / W + j * (kWave + kWave / W);
        } else {
            const int e = lane + kWave * j;
            return e + e / W;
        }
    }

    template <int W>
    __device__ __forceinline__ void gather(const double *g, double (&c)[W]) const {
        const double *base = g + first * W;
        const int lim = nvalid * W;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int e = lane + kWave * j;
            c[j] = e < lim ? base[e] : 0.0;
        }
    }

    template <int W>
    __device__ __forceinline__ void to_lanes(const double (&c)[W], double (&v)[W]) const {
        if constexpr (W == 1) {
            v[0] = c[0];
        } else {
            order();
#pragma unroll
            for (int j = 0; j < W; ++j) lds[slot<W>(j)] = c[j];
            order();
#pragma unroll
            for (int k = 0; k < W; ++k) v[k] = lds[lane * tile_stride<W>() + k];
            order();
        }
    }

    template <int W>
    __device__ __forceinline__ void load(const double *g, double (&v)[W]) const {
        double c[W];
        gather<W>(g, c);
        to_lanes<W>(c, v);
    }

    template <int W>
    __device__ __forceinline__ void from_lanes(const double (&v)[W], double (&c)[W]) const {
        if constexpr (W == 1) {
            c[0] = v[0];
        } else {
            order();
#pragma unroll
            for (int k = 0; k < W; ++k) lds[lane * tile_stride<W>() + k] = v[k];
            order();
#pragma unroll
            for (int j = 0; j < W; ++j) c[j] = lds[slot<W>(j)];
            order();
        }
    }

    template <int W>
    __device__ __forceinline__ void scatter(double *g, const double (&c)[W]) const {
        double *base = g + first * W;
        const int lim = nvalid * W;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int e = lane + kWave * j;
            if (e < lim) base[e] = c[j];
        }
    }

    template <int W>
    __device__ __forceinline__ void store(double *g, const double (&v)[W]) const {
        double c[W];
        from_lanes<W>(v, c);
        scatter<W>(g, c);
    }
};

}  // namespace pekf
