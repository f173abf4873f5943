// rccl_selftest: one-rank RCCL communicator on device 0 — bootstrap, an 8-byte all-reduce and a
// grouped self send/recv of one p = 2 interface plane (the calls csrc/comm.hip issues on slabs).
// Built by the package Makefile into lib/rccl_selftest; run by tests/test_gpu_rccl.py.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <vector>

#define NC(x)                                                                                  \
    do {                                                                                       \
        ncclResult_t r_ = (x);                                                                 \
        if (r_ != ncclSuccess) {                                                               \
            std::printf("FAIL %s: %d %s\n", #x, (int)r_, ncclGetErrorString(r_));              \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)
#define HC(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                           \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

int main()
{
    int ver = 0;
    NC(ncclGetVersion(&ver));
    std::printf("rccl version %d\n", ver);
    HC(hipSetDevice(0));
    ncclUniqueId id;
    NC(ncclGetUniqueId(&id));
    ncclComm_t comm;
    NC(ncclCommInitRank(&comm, 1, id, 0));
    std::printf("init ok\n");
    hipStream_t s;
    HC(hipStreamCreate(&s));
    const int n = 129 * 129;
    std::vector<double> a(n), b(n, 0.0);
    for (int i = 0; i < n; ++i) a[i] = 0.001 * i - 3.0;
    double *da, *db, *dr;
    HC(hipMalloc(&da, n * 8));
    HC(hipMalloc(&db, n * 8));
    HC(hipMalloc(&dr, 8));
    const double red = 3.25;
    HC(hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(dr, &red, 8, hipMemcpyHostToDevice));
    NC(ncclAllReduce(dr, dr, 1, ncclDouble, ncclSum, comm, s));
    NC(ncclGroupStart());
    NC(ncclSend(da, n, ncclDouble, 0, comm, s));
    NC(ncclRecv(db, n, ncclDouble, 0, comm, s));
    NC(ncclGroupEnd());
    HC(hipStreamSynchronize(s));
    double got = 0.0;
    HC(hipMemcpy(&got, dr, 8, hipMemcpyDeviceToHost));
    HC(hipMemcpy(b.data(), db, n * 8, hipMemcpyDeviceToHost));
    int bad = got != red;
    for (int i = 0; i < n; ++i) bad += b[i] != a[i];
    std::printf("allreduce %.17g, mismatches %d\n", got, bad);
    NC(ncclCommDestroy(comm));
    HC(hipStreamDestroy(s));
    std::printf(bad ? "RCCL SELFTEST FAIL\n" : "RCCL SELFTEST OK\n");
    return bad ? 1 : 0;
}
