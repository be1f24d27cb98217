// ci_kernels.hip -- batched G^2 conditional-independence tests on gfx950.
//
// One 256-thread workgroup per test (grid-stride over the batch).  The column store is uint8
// [var][sample]; each thread streams 4 samples per load (one dword per column) and bins them into
// the contingency table N[z][x][y] held in LDS with LDS atomics (small tables are first reduced
// inside the wave with ballots, which avoids 64-way same-address conflicts).  Marginals, the
// adjusted degrees of freedom and the G^2 terms are then evaluated per z-configuration by
// parallel threads, summed in z order, and one lane evaluates p = Q(df/2, G^2/2).
//
// Reference: Counts2D/Counts3D (src/CellTable.cpp:23-91,226-291,430-455) and
// ComputeGSquareXY/XYZ (src/IndependenceTest.cpp:65-155,295-364).  Counts and df are exact;
// G^2 is summed per z then across z (vs one running sum in the reference): <= a few ulp apart.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct CiArgs {
    const uint8_t *cols;  // [nvars][N]
    const int32_t *dims;
    const int32_t *items;  // [n][2+D]
    long long N;
    long long n;
    double alpha;
    double *g2;
    int32_t *df;
    double *p;
    uint8_t *indep;
    int32_t *counts;  // optional: histogram of item 0
};

// regularized upper incomplete gamma Q(a, x): series / modified Lentz continued fraction; the
// same algorithm as the oracle restatement of stats::pchisq (oracle/pc_oracle.cpp)
__device__ double gamma_q(double a, double x) {
    if (x <= 0.0) return 1.0;
    const double lg = lgamma(a);
    if (x < a + 1.0) {
        double ap = a, sum = 1.0 / a, del = sum;
        for (int n = 0; n < 2000; ++n) {
            ap += 1.0;
            del *= x / ap;
            sum += del;
            if (fabs(del) < fabs(sum) * 1e-17) break;
        }
        return 1.0 - sum * exp(-x + a * log(x) - lg);
    }
    const double tiny = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
    for (int i = 1; i < 2000; ++i) {
        const double an = -i * (i - a);
        b += 2.0;
        d = an * d + b;
        if (fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < 1e-17) break;
    }
    return exp(-x + a * log(x) - lg) * h;
}

template <int D>
__global__ __launch_bounds__(256) void ci_g2_kernel(CiArgs A) {
    extern __shared__ __align__(16) int32_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    for (long long it = blockIdx.x; it < A.n; it += gridDim.x) {
        const int32_t *item = A.items + it * (2 + D);
        const int x = item[0], y = item[1];
        const int dx = A.dims[x], dy = A.dims[y];
        int zv[D > 0 ? D : 1], cum[D > 0 ? D : 1];
        int dimz = 1;
#pragma unroll
        for (int j = D - 1; j >= 0; --j) {
            zv[j] = item[2 + j];
            cum[j] = dimz;  // last conditioning variable fastest (src/CellTable.cpp:39-51)
            dimz *= A.dims[zv[j]];
        }
        const int dxy = dx * dy;
        const int cells = dimz * dxy;
        int32_t *hist = smem;
        int32_t *ni = hist + cells;
        int32_t *nj = ni + dimz * dx;
        int32_t *nk = nj + dimz * dy;
        int32_t *dfp = nk + dimz;
        double *part = reinterpret_cast<double *>(smem + ((cells + dimz * (dx + dy + 2) + 1) & ~1));

        for (int c = tid; c < cells; c += 256) hist[c] = 0;
        __syncthreads();

        const uint8_t *cx = A.cols + (size_t)x * A.N;
        const uint8_t *cy = A.cols + (size_t)y * A.N;
        const uint8_t *cz[D > 0 ? D : 1];
#pragma unroll
        for (int j = 0; j < D; ++j) cz[j] = A.cols + (size_t)zv[j] * A.N;

        const bool small = cells <= 32;
        auto bin = [&](int cell, bool valid) {
            if (small) {
                // wave-aggregated: one LDS add per distinct cell present in the wave
                unsigned long long todo = __ballot(valid);
                while (todo) {
                    const int leader = __ffsll(todo) - 1;
                    const int lc = __shfl(cell, leader);
                    const unsigned long long same = __ballot(valid && cell == lc);
                    if (lane == leader) atomicAdd(&hist[lc], __popcll(same));
                    todo &= ~same;
                }
            } else if (valid) {
                atomicAdd(&hist[cell], 1);
            }
        };
        const long long N4 = (A.N % 4 == 0) ? A.N / 4 : 0;
        for (long long k4 = tid; k4 < ((N4 + 255) / 256) * 256; k4 += 256) {
            const bool v4 = k4 < N4;
            uint32_t wx = 0, wy = 0, wz[D > 0 ? D : 1];
            if (v4) {
                wx = reinterpret_cast<const uint32_t *>(cx)[k4];
                wy = reinterpret_cast<const uint32_t *>(cy)[k4];
            }
#pragma unroll
            for (int j = 0; j < D; ++j) wz[j] = v4 ? reinterpret_cast<const uint32_t *>(cz[j])[k4] : 0u;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                int zi = 0;
#pragma unroll
                for (int j = 0; j < D; ++j) zi += (int)((wz[j] >> (8 * s)) & 0xFF) * cum[j];
                const int cell = (zi * dx + (int)((wx >> (8 * s)) & 0xFF)) * dy + (int)((wy >> (8 * s)) & 0xFF);
                bin(cell, v4);
            }
        }
        for (long long k = 4 * N4 + tid; k < ((A.N - 4 * N4 + 255) / 256) * 256 + 4 * N4; k += 256) {
            const bool v = k < A.N;
            int cell = 0;
            if (v) {
                int zi = 0;
#pragma unroll
                for (int j = 0; j < D; ++j) zi += (int)cz[j][k] * cum[j];
                cell = (zi * dx + cx[k]) * dy + cy[k];
            }
            bin(cell, v);
        }
        __syncthreads();
        if (A.counts && it == 0)
            for (int c = tid; c < cells; c += 256) A.counts[c] = hist[c];

        // marginals N_{x+z}, N_{+yz}, N_{++z} (src/CellTable.cpp:242-250)
        for (int r = tid; r < dimz * dx; r += 256) {
            const int k = r / dx, i = r % dx;
            int s = 0;
            for (int j = 0; j < dy; ++j) s += hist[k * dxy + i * dy + j];
            ni[r] = s;
        }
        for (int r = tid; r < dimz * dy; r += 256) {
            const int k = r / dy, j = r % dy;
            int s = 0;
            for (int i = 0; i < dx; ++i) s += hist[k * dxy + i * dy + j];
            nj[r] = s;
        }
        __syncthreads();
        // per z: adjusted df and G^2 terms in the reference's i -> j order
        for (int k = tid; k < dimz; k += 256) {
            int alx = 0, aly = 0;
            long total = 0;
            for (int i = 0; i < dx; ++i) alx += ni[k * dx + i] > 0, total += ni[k * dx + i];
            for (int j = 0; j < dy; ++j) aly += nj[k * dy + j] > 0;
            alx = alx >= 1 ? alx : 1;
            aly = aly >= 1 ? aly : 1;
            dfp[k] = (alx - 1) * (aly - 1);
            double g = 0.0;
            if (total != 0) {
                for (int i = 0; i < dx; ++i) {
                    const long sum_row = ni[k * dx + i];
                    if (sum_row == 0) continue;
                    for (int j = 0; j < dy; ++j) {
                        const long sum_col = nj[k * dy + j];
                        const long observed = hist[k * dxy + i * dy + j];
                        if (sum_col == 0 || observed == 0) continue;
                        const double expected = (double)sum_col * (double)sum_row / (double)total;
                        g += 2.0 * observed * log(observed / expected);
                    }
                }
            }
            part[k] = g;
        }
        __syncthreads();
        if (tid == 0) {
            double g2 = 0.0;
            int df = 0;
            for (int k = 0; k < dimz; ++k) g2 += part[k], df += dfp[k];
            double p;
            bool ind;
            if (df == 0) {  // src/IndependenceTest.cpp:149-151, 349-351
                p = 1.0;
                ind = true;
            } else {
                p = gamma_q(0.5 * df, 0.5 * g2);
                ind = p > A.alpha;
            }
            if (A.g2) A.g2[it] = g2;
            if (A.df) A.df[it] = df;
            if (A.p) A.p[it] = p;
            if (A.indep) A.indep[it] = ind;
        }
        __syncthreads();
    }
}

}  // namespace

// LDS bytes needed for a test with `cells` = dimz*dx*dy
extern "C" size_t fbn_ci_lds_bytes(int dimz, int dx, int dy) {
    size_t ints = (size_t)dimz * dx * dy + (size_t)dimz * (dx + dy + 2) + 1;
    ints = (ints + 1) & ~(size_t)1;
    return ints * 4 + (size_t)dimz * 8;
}

extern "C" hipError_t fbn_ci_launch(const uint8_t *cols, const int32_t *dims, const int32_t *items, long long N,
                                    long long n, int d, double alpha, double *g2, int32_t *df, double *p,
                                    uint8_t *indep, int32_t *counts, size_t lds_bytes, int grid,
                                    hipStream_t stream) {
    CiArgs a{cols, dims, items, N, n, alpha, g2, df, p, indep, counts};
    switch (d) {
#define FBN_CI_CASE(DD)                                                                              \
    case DD:                                                                                         \
        hipLaunchKernelGGL(ci_g2_kernel<DD>, dim3(grid), dim3(256), lds_bytes, stream, a);           \
        break;
        FBN_CI_CASE(0)
        FBN_CI_CASE(1)
        FBN_CI_CASE(2)
        FBN_CI_CASE(3)
        FBN_CI_CASE(4)
        FBN_CI_CASE(5)
        FBN_CI_CASE(6)
        FBN_CI_CASE(7)
        FBN_CI_CASE(8)
#undef FBN_CI_CASE
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
