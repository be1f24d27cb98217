// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the JT kernel's access width (8 B per lane,
// 512 B per wave instruction): copy 512 MiB with global_load/store_dwordx2 (grid-stride).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void copy8(const double *__restrict__ a, double *__restrict__ b, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = a[i] + 1.0;
}

int main() {
    const long long n = (512ll << 20) / 8;
    double *a, *b;
    if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess) return 1;
    (void)hipMemset(a, 0, n * 8);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(copy8, dim3(4096), dim3(256), 0, 0, a, b, n);
    (void)hipDeviceSynchronize();
    printf("copy8: %lld bytes read + %lld bytes written per launch\n", n * 8, n * 8);
    return 0;
}
