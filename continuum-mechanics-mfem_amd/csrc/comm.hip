// comm.hip — rank communication for the element-partitioned (slab) multi-GPU path.
//
// Replaces the reference's MPI layer on the hot path (SURVEY.md §5 "Distributed comm backend"):
// ParMesh(MPI_COMM_WORLD) element partition (linear_convection_diffusion_2D.cpp:300), hypre/PETSc
// halo exchange inside MatMult and the MPI_Allreduce of the Krylov dot products.
//
// Each rank owns a z-slab of the structured box.  Its local L-vector holds the dofs of its
// elements; the interface planes (local gz = 0 / gz = Lz-1) are shared with the rank below / above
// and are OWNED by the lower rank for dot products.  Per Krylov iteration:
//   * the two interface planes' LOCAL partial sums of q = A d are exchanged with the neighbours
//     (RCCL send/recv, 8*(p nx + 1)*(p ny + 1) bytes per plane) and added by the update kernel;
//   * the three Krylov scalars (nom, den, betanom) are summed with an 8-byte all-reduce.
// Two backends: RCCL (stream-ordered, no host sync: the production path over xGMI) and host
// callbacks (device->host staging + user functions, e.g. torch.distributed/gloo or MPI; used to
// test the distributed kernels with several processes on ONE GPU, which RCCL refuses).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "cdfem_internal.hpp"

namespace cdfem {

struct Comm {
    int rank = 0, nranks = 1;
    ncclComm_t nccl = nullptr;
    cdfem_allreduce_fn h_allreduce = nullptr;
    cdfem_exchange_fn h_exchange = nullptr;
    void *user = nullptr;
    cdfem_nbr_exchange_fn h_nbr = nullptr;  // general partition (host backend)
    void *nbr_user = nullptr;
    double *h_buf = nullptr;  // pinned staging for the host backend
    size_t h_cap = 0;
    int refs = 1;             // contexts using this communicator (cdfem_comm_share)
};

static void nccl_check(ncclResult_t r, const char *what)
{
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

void comm_destroy(cdfem_ctx *c)
{
    if (!c->comm) return;
    if (--c->comm->refs == 0) {
        if (c->comm->nccl) (void)ncclCommDestroy(c->comm->nccl);
        if (c->comm->h_buf) (void)hipHostFree(c->comm->h_buf);
        delete c->comm;
    }
    c->comm = nullptr;
    c->rank = 0;
    c->nranks = 1;
}

static double *host_staging(Comm *m, size_t n)
{
    if (m->h_cap < n) {
        if (m->h_buf) (void)hipHostFree(m->h_buf);
        if (hipHostMalloc(&m->h_buf, n * sizeof(double), hipHostMallocDefault) != hipSuccess)
            throw std::runtime_error("pinned staging allocation failed");
        m->h_cap = n;
    }
    return m->h_buf;
}

// in-place sum over ranks of n doubles in device memory (stream-ordered)
void comm_allreduce(cdfem_ctx *c, double *dbuf, int n)
{
    Comm *m = c->comm;
    if (!m || m->nranks == 1) return;
    if (m->nccl) {
        nccl_check(ncclAllReduce(dbuf, dbuf, n, ncclDouble, ncclSum, m->nccl, c->stream), "ncclAllReduce");
        return;
    }
    double *h = host_staging(m, n);
    if (hipMemcpyAsync(h, dbuf, n * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        throw std::runtime_error("allreduce staging failed");
    if (m->h_allreduce(h, n, m->user) != 0) throw std::runtime_error("host allreduce callback failed");
    // the staging buffer may be shared with other contexts (cdfem_comm_share): complete the
    // upload before any other exchange can overwrite it
    if (hipMemcpyAsync(dbuf, h, n * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        throw std::runtime_error("allreduce staging failed");
}

// exchange interface planes with the neighbours: send_lo -> rank-1 (recv into its recv_hi) and
// send_hi -> rank+1; n doubles per plane
void comm_exchange(cdfem_ctx *c, const double *send_lo, double *recv_lo, const double *send_hi,
                   double *recv_hi, int64_t n, hipStream_t s)
{
    if (!s) s = c->stream;
    Comm *m = c->comm;
    if (!m || m->nranks == 1) return;
    // the neighbours are the ones the slab declared (cdfem_set_slab), not the rank arithmetic
    const bool lo = c->zlo_shared != 0, hi = c->zhi_shared != 0;
    if ((lo && m->rank == 0) || (hi && m->rank == m->nranks - 1))
        throw std::runtime_error("slab declares a neighbour rank that does not exist");
    if (m->nccl) {
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        if (lo) {
            nccl_check(ncclSend(send_lo, n, ncclDouble, m->rank - 1, m->nccl, s), "ncclSend");
            nccl_check(ncclRecv(recv_lo, n, ncclDouble, m->rank - 1, m->nccl, s), "ncclRecv");
        }
        if (hi) {
            nccl_check(ncclSend(send_hi, n, ncclDouble, m->rank + 1, m->nccl, s), "ncclSend");
            nccl_check(ncclRecv(recv_hi, n, ncclDouble, m->rank + 1, m->nccl, s), "ncclRecv");
        }
        nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        return;
    }
    double *h = host_staging(m, 4 * (size_t)n);
    double *hs_lo = h, *hr_lo = h + n, *hs_hi = h + 2 * n, *hr_hi = h + 3 * n;
    if ((lo && hipMemcpyAsync(hs_lo, send_lo, n * 8, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (hi && hipMemcpyAsync(hs_hi, send_hi, n * 8, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess)
        throw std::runtime_error("exchange staging failed");
    if (m->h_exchange(lo ? hs_lo : nullptr, lo ? hr_lo : nullptr, hi ? hs_hi : nullptr,
                      hi ? hr_hi : nullptr, n, m->user) != 0)
        throw std::runtime_error("host exchange callback failed");
    if ((lo && hipMemcpyAsync(recv_lo, hr_lo, n * 8, hipMemcpyHostToDevice, s) != hipSuccess) ||
        (hi && hipMemcpyAsync(recv_hi, hr_hi, n * 8, hipMemcpyHostToDevice, s) != hipSuccess))
        throw std::runtime_error("exchange staging failed");
    // the staging buffer is reused by the next call: complete the uploads first
    if (hipStreamSynchronize(s) != hipSuccess) throw std::runtime_error("exchange staging failed");
}

// ---- plane kernels ----------------------------------------------------------------------------
__global__ void k_get_plane(const double *__restrict__ v, int64_t plane_off, int64_t n,
                            double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v[plane_off + i];
}

__global__ void k_add_plane(double *__restrict__ v, int64_t plane_off, int64_t n,
                            const double *__restrict__ in)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[plane_off + i] += in[i];
}

__global__ void k_copy_plane(double *__restrict__ v, int64_t plane_off, int64_t n, const double *__restrict__ in)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[plane_off + i] = in[i];
}

// ---- general partition (cdfem_set_shared) ---------------------------------------------------------
__global__ void k_sh_pack(const double *__restrict__ v, const int32_t *__restrict__ idx, int64_t n,
                          double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = v[idx[i]];
}

// v[d] = sum of every holder's partial in ascending rank order (own partial at src = -1): every
// rank forms the same sum in the same order, so all copies of a shared dof are bitwise equal
__global__ void k_sh_sum(double *__restrict__ v, const int32_t *__restrict__ dofs, const int32_t *__restrict__ off,
                         const int32_t *__restrict__ src, int32_t n, const double *__restrict__ recv)
{
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t d = dofs[i];
    const double own = v[d];
    double acc = 0.0;
    for (int32_t k = off[i]; k < off[i + 1]; ++k) {
        const int32_t s = src[k];
        acc += s < 0 ? own : recv[s];
    }
    v[d] = acc;
}

// non-owned shared dofs take the owner's copy
__global__ void k_sh_copy_owner(double *__restrict__ v, const int32_t *__restrict__ dofs,
                                const int32_t *__restrict__ owner, int32_t n, const double *__restrict__ recv)
{
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && owner[i] >= 0) v[dofs[i]] = recv[owner[i]];
}

// send[off[k]..off[k+1]) -> nbr_rank[k], recv[same range] <- nbr_rank[k], for every neighbour
// (device buffers; the two ranks of a pair use the same count)
void comm_exchange_nbr_buf(cdfem_ctx *c, const std::vector<int64_t> &off, const double *dsend, double *drecv,
                           hipStream_t s)
{
    if (!s) s = c->stream;
    Comm *m = c->comm;
    const int nn = (int)c->nbr_rank.size();
    if (nn == 0 || !m || m->nranks == 1) return;
    const int64_t ntot = off[nn];
    if (m->nccl) {
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        for (int k = 0; k < nn; ++k) {
            const int64_t o = off[k], cnt = off[k + 1] - o;
            nccl_check(ncclSend(dsend + o, cnt, ncclDouble, c->nbr_rank[k], m->nccl, s), "ncclSend");
            nccl_check(ncclRecv(drecv + o, cnt, ncclDouble, c->nbr_rank[k], m->nccl, s), "ncclRecv");
        }
        nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        return;
    }
    if (!m->h_nbr) throw std::runtime_error("host communicator has no neighbour exchange (cdfem_comm_set_host_nbr_exchange)");
    double *h = host_staging(m, 2 * (size_t)ntot);
    if (hipMemcpyAsync(h, dsend, ntot * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        throw std::runtime_error("exchange staging failed");
    if (m->h_nbr(nn, c->nbr_rank.data(), off.data(), h, h + ntot, m->nbr_user) != 0)
        throw std::runtime_error("host neighbour exchange callback failed");
    if (hipMemcpyAsync(drecv, h + ntot, ntot * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        throw std::runtime_error("exchange staging failed");
}

static void comm_exchange_nbr(cdfem_ctx *c, hipStream_t s)
{
    if (c->nbr_rank.empty()) return;
    comm_exchange_nbr_buf(c, c->nbr_off, c->d_sh_send, c->d_sh_recv, s);
}

static void shared_pack_exchange(cdfem_ctx *c, const double *v)
{
    const int64_t ntot = c->nbr_off.empty() ? 0 : c->nbr_off.back();
    if (ntot > 0)
        hipLaunchKernelGGL(k_sh_pack, dim3((unsigned)((ntot + 255) / 256)), dim3(256), 0, c->stream, v, c->d_sh_idx,
                           ntot, c->d_sh_send);
    comm_exchange_nbr(c, c->stream);
}

void partition_free(cdfem_ctx *c)
{
    for (int32_t **p : {&c->d_sh_idx, &c->d_shd, &c->d_shd_off, &c->d_shd_src, &c->d_shd_owner}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    for (double **p : {&c->d_sh_send, &c->d_sh_recv}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    c->nbr_rank.clear();
    c->nbr_off.clear();
    c->h_sh_idx.clear();
    ilu_free(c);  // a block-Jacobi factor belongs to the previous partition
    c->n_shd = 0;
    c->part_mode = 0;
    c->skip_lo = 0;
}

// non-owned shared entries <- the owner's value (slab: the lower plane from the rank below)
void interface_copy_owner(cdfem_ctx *c, double *v)
{
    if (!c->comm || c->comm->nranks == 1) return;
    if (c->part_mode == 2) {
        shared_pack_exchange(c, v);
        if (c->n_shd > 0)
            hipLaunchKernelGGL(k_sh_copy_owner, dim3((unsigned)((c->n_shd + 255) / 256)), dim3(256), 0, c->stream, v,
                               c->d_shd, c->d_shd_owner, c->n_shd, c->d_sh_recv);
        return;
    }
    if (c->part_mode != 1) return;
    const int64_t n = c->Lx * c->Ly, off_hi = (c->Lz - 1) * n;
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    if (c->zlo_shared) hipLaunchKernelGGL(k_get_plane, g, b, 0, c->stream, v, (int64_t)0, n, c->d_if[0]);
    if (c->zhi_shared) hipLaunchKernelGGL(k_get_plane, g, b, 0, c->stream, v, off_hi, n, c->d_if[2]);
    comm_exchange(c, c->d_if[0], c->d_if[1], c->d_if[2], c->d_if[3], n);
    if (c->zlo_shared) hipLaunchKernelGGL(k_copy_plane, g, b, 0, c->stream, v, (int64_t)0, n, c->d_if[1]);
}

// sum of the interface planes of an L-vector over the ranks sharing them (MFEM P^T then P)
void interface_sum(cdfem_ctx *c, double *v)
{
    if (!c->comm || c->comm->nranks == 1) return;
    if (c->part_mode == 2) {
        shared_pack_exchange(c, v);
        if (c->n_shd > 0)
            hipLaunchKernelGGL(k_sh_sum, dim3((unsigned)((c->n_shd + 255) / 256)), dim3(256), 0, c->stream, v, c->d_shd,
                               c->d_shd_off, c->d_shd_src, c->n_shd, c->d_sh_recv);
        return;
    }
    if (c->part_mode != 1) return;
    const int64_t n = c->Lx * c->Ly, off_hi = (c->Lz - 1) * n;
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    if (c->zlo_shared) hipLaunchKernelGGL(k_get_plane, g, b, 0, c->stream, v, (int64_t)0, n, c->d_if[0]);
    if (c->zhi_shared) hipLaunchKernelGGL(k_get_plane, g, b, 0, c->stream, v, off_hi, n, c->d_if[2]);
    comm_exchange(c, c->d_if[0], c->d_if[1], c->d_if[2], c->d_if[3], n);
    if (c->zlo_shared) hipLaunchKernelGGL(k_add_plane, g, b, 0, c->stream, v, (int64_t)0, n, c->d_if[1]);
    if (c->zhi_shared) hipLaunchKernelGGL(k_add_plane, g, b, 0, c->stream, v, off_hi, n, c->d_if[3]);
}

}  // namespace cdfem

using namespace cdfem;

extern "C" {

int cdfem_comm_unique_id(unsigned char *id)
{
    if (!id) return CDFEM_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return CDFEM_ERR_COMM;
    for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) id[i] = (unsigned char)u.internal[i];
    return CDFEM_OK;
}

int cdfem_comm_init_rccl(cdfem_ctx *c, int rank, int nranks, const unsigned char *id)
{
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return CDFEM_ERR_ARG;
    comm_destroy(c);
    Comm *m = new Comm();
    m->rank = rank;
    m->nranks = nranks;
    {
        // a one-rank communicator is created too (its collectives are never issued: every
        // exchange returns early at nranks == 1); tests/test_gpu_rccl.py initialises one beside a
        // live context, as every rank of the N > 1 bench does
        ncclUniqueId u;
        for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) u.internal[i] = (char)id[i];
        if (hipSetDevice(c->device) != hipSuccess) {
            delete m;
            return CDFEM_ERR_HIP;
        }
        const ncclResult_t r = ncclCommInitRank(&m->nccl, nranks, u, rank);
        if (r != ncclSuccess) {
            c->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            delete m;
            return CDFEM_ERR_COMM;
        }
    }
    c->comm = m;
    c->rank = rank;
    c->nranks = nranks;
    return CDFEM_OK;
}

int cdfem_comm_set_host_nbr_exchange(cdfem_ctx *c, cdfem_nbr_exchange_fn fn, void *user)
{
    if (!c || !fn) return CDFEM_ERR_ARG;
    if (!c->comm || c->comm->nccl) {
        c->err = "cdfem_comm_set_host_nbr_exchange: attach a host communicator first (cdfem_comm_init_host)";
        return CDFEM_ERR_STATE;
    }
    c->comm->h_nbr = fn;
    c->comm->nbr_user = user;
    return CDFEM_OK;
}

int cdfem_comm_share(cdfem_ctx *dst, const cdfem_ctx *src)
{
    if (!dst || !src || dst == src) return CDFEM_ERR_ARG;
    if (!src->comm) {
        dst->err = "cdfem_comm_share: the source context has no communicator";
        return CDFEM_ERR_STATE;
    }
    if (src->comm->nccl && src->device != dst->device) {
        dst->err = "cdfem_comm_share: an RCCL communicator is bound to the source context's device";
        return CDFEM_ERR_ARG;
    }
    comm_destroy(dst);
    dst->comm = src->comm;
    dst->comm->refs++;
    dst->rank = src->rank;
    dst->nranks = src->nranks;
    return CDFEM_OK;
}

int cdfem_comm_info(const cdfem_ctx *c, char *buf, size_t n)
{
    if (!buf || n == 0) return CDFEM_ERR_ARG;
    int v = 0;
    (void)ncclGetVersion(&v);
    Dl_info info{};
    const char *path = dladdr(reinterpret_cast<void *>(&ncclGetVersion), &info) && info.dli_fname
                           ? info.dli_fname : "?";
    const char *backend = !c || !c->comm ? "none" : c->comm->nccl ? "rccl" : "host";
    const int w = std::snprintf(buf, n, "backend=%s rccl_version=%d rccl_path=%s", backend, v, path);
    return (w < 0 || (size_t)w >= n) ? CDFEM_ERR_ARG : CDFEM_OK;
}

int cdfem_comm_init_host(cdfem_ctx *c, int rank, int nranks, cdfem_allreduce_fn allreduce,
                         cdfem_exchange_fn exchange, void *user)
{
    if (!c || !allreduce || !exchange || nranks < 1 || rank < 0 || rank >= nranks) return CDFEM_ERR_ARG;
    comm_destroy(c);
    Comm *m = new Comm();
    m->rank = rank;
    m->nranks = nranks;
    m->h_allreduce = allreduce;
    m->h_exchange = exchange;
    m->user = user;
    c->comm = m;
    c->rank = rank;
    c->nranks = nranks;
    return CDFEM_OK;
}

}  // extern "C"
