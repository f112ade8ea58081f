/*
 * Key extraction on the device: a stream of pipelined
 * memcache retrieval requests ("get k1 k2 ...\r\n", "gets ...\r\n") into the
 * key CSR the hash kernels take, plus the request each key belongs to.
 *
 * Reference: memcache_parse_req, /root/reference/src/proto/nc_memcache.c,
 * for the retrieval commands:
 *   - SW_START (:219-232): leading spaces, then a lowercase letter;
 *   - SW_REQ_TYPE (:234-368): lowercase letters up to ' ' or CR; "get" (:245)
 *     and "gets" (:268) are the retrieval types; a CR right after them is an
 *     error (:343-345);
 *   - SW_SPACES_BEFORE_KEY (:372-378), SW_KEY (:380-428): a key is every byte
 *     up to ' ' or CR; length 0 or > MEMCACHE_MAX_KEY_LENGTH (250, :33) is an
 *     error (:384-396);
 *   - SW_SPACES_BEFORE_KEYS (:431-447): spaces, CR ends the key list;
 *   - SW_ALMOST_DONE (:709-717): CR must be followed by LF.
 * The reference parses sequentially and closes the connection at the first
 * bad request; here every complete line ("...\r\n") is parsed in parallel and
 * keys are emitted for the requests before the first bad one, i.e. exactly
 * what the reference accepts before it errors. Any other command ends the
 * parsable prefix too (its data block, for storage commands, is not a line):
 * the caller hands the rest to the host parser.
 *
 * Device steps: mark LFs that follow a CR -> compact their positions
 * (hipCUB DeviceSelect) -> one thread per line parses it (status, key count,
 * first error via atomicMin) -> exclusive scan of key counts -> a second
 * parse writes each key's (start, length, request) -> exclusive scan of
 * lengths -> one thread per key copies its bytes into the packed CSR.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <errno.h>
#include <stdlib.h>

#include "nc_gpuhash.h"

namespace {

constexpr uint32_t kMaxKeyLen = 250; /* MEMCACHE_MAX_KEY_LENGTH, nc_memcache.c:33 */

struct Line {
    uint64_t start, cr; /* [start, cr): the request; cr = position of its CR */
};

__device__ __forceinline__ Line line_of(const uint64_t *__restrict__ lf, uint64_t r)
{
    Line l;
    l.start = r == 0 ? 0u : lf[r - 1] + 1u;
    l.cr = lf[r] - 1u;
    return l;
}

/* The state machine of one request line. EMIT = false: count keys and
 * validate; EMIT = true: also write each key's span. Returns the status. */
template <bool EMIT>
__device__ int32_t parse_line(const uint8_t *__restrict__ s, Line l, uint32_t *nkeys, uint64_t *kstart,
                              uint32_t *klen, uint32_t *kreq, uint64_t base, uint32_t req)
{
    uint64_t p = l.start;
    while (p < l.cr && s[p] == ' ') p++;                       /* SW_START */
    const uint64_t t0 = p;
    while (p < l.cr && s[p] >= 'a' && s[p] <= 'z') p++;       /* SW_REQ_TYPE */
    const uint64_t tl = p - t0;
    if (tl == 0 || (p < l.cr && s[p] != ' ')) return NC_GPUHASH_MC_EINVAL; /* not a lowercase type */
    const bool get = tl == 3 && s[t0] == 'g' && s[t0 + 1] == 'e' && s[t0 + 2] == 't';
    const bool gets = tl == 4 && s[t0] == 'g' && s[t0 + 1] == 'e' && s[t0 + 2] == 't' && s[t0 + 3] == 's';
    if (!get && !gets) return NC_GPUHASH_MC_EUNSUPPORTED; /* the host parser takes over */
    if (p == l.cr) return NC_GPUHASH_MC_EINVAL;            /* "get\r\n" (nc_memcache.c:343-345) */
    uint32_t n = 0;
    while (p < l.cr && s[p] == ' ') p++;                       /* SW_SPACES_BEFORE_KEY */
    for (;;) {
        if (p < l.cr && s[p] == '\r') return NC_GPUHASH_MC_EINVAL; /* CR not followed by LF */
        const uint64_t k0 = p;                                /* SW_KEY: up to ' ' or CR */
        while (p < l.cr && s[p] != ' ' && s[p] != '\r') p++;
        const uint64_t len = p - k0;
        if (len == 0 || len > kMaxKeyLen) return NC_GPUHASH_MC_EKEYLEN;
        if constexpr (EMIT) {
            kstart[base + n] = k0;
            klen[base + n] = (uint32_t)len;
            kreq[base + n] = req;
        }
        n++;
        if (p < l.cr && s[p] == '\r') return NC_GPUHASH_MC_EINVAL; /* CR not followed by LF */
        while (p < l.cr && s[p] == ' ') p++;                   /* SW_SPACES_BEFORE_KEYS */
        if (p == l.cr) break;                                 /* CR LF: done (SW_ALMOST_DONE) */
    }
    *nkeys = n;
    return NC_GPUHASH_MC_OK;
}

__global__ void mc_mark_kernel(const uint8_t *__restrict__ s, uint64_t nbytes, uint8_t *__restrict__ flag)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nbytes; i += (uint64_t)gridDim.x * 256u)
        flag[i] = (i > 0 && s[i] == '\n' && s[i - 1] == '\r') ? 1u : 0u;
}

__global__ void mc_count_kernel(const uint8_t *__restrict__ s, const uint64_t *__restrict__ lf, uint64_t nreq,
                                int32_t *__restrict__ status, uint32_t *__restrict__ nkeys,
                                unsigned long long *__restrict__ first_bad)
{
    const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (r >= nreq) return;
    uint32_t n = 0;
    const int32_t st = parse_line<false>(s, line_of(lf, r), &n, nullptr, nullptr, nullptr, 0, 0);
    status[r] = st;
    nkeys[r] = st == 0 ? n : 0u;
    if (st != 0) atomicMin(first_bad, (unsigned long long)r);
}

__global__ void mc_clip_kernel(uint32_t *__restrict__ nkeys, uint64_t nreq, const unsigned long long *first_bad)
{
    const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (r < nreq && r >= *first_bad) nkeys[r] = 0u;
}

__global__ void mc_emit_kernel(const uint8_t *__restrict__ s, const uint64_t *__restrict__ lf, uint64_t nreq,
                               const unsigned long long *first_bad, const uint64_t *__restrict__ kbase,
                               uint64_t *__restrict__ kstart, uint32_t *__restrict__ klen, uint32_t *__restrict__ kreq)
{
    const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (r >= nreq || r >= *first_bad) return;
    uint32_t n = 0;
    (void)parse_line<true>(s, line_of(lf, r), &n, kstart, klen, kreq, kbase[r], (uint32_t)r);
}

__global__ void mc_gather_kernel(const uint8_t *__restrict__ s, const uint64_t *__restrict__ kstart,
                                 const uint64_t *__restrict__ koff, uint64_t nk, uint8_t *__restrict__ keys)
{
    const uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (k >= nk) return;
    const uint64_t src = kstart[k], dst = koff[k], len = koff[k + 1] - koff[k];
    for (uint64_t j = 0; j < len; j++) keys[dst + j] = s[src + j];
}

__global__ void mc_pad_kernel(uint8_t *__restrict__ keys, const uint64_t *__restrict__ koff, uint64_t nk)
{
    const uint64_t e = koff[nk];
    if (threadIdx.x < NC_GPUHASH_PAD) keys[e + threadIdx.x] = 0u;
}

/* length u32 -> u64 for the offsets scan */
struct Widen {
    __host__ __device__ uint64_t operator()(uint32_t v) const { return v; }
};

/* one thread per item: n < 2^31 (the workspace limit), so n / 256 blocks fit */
unsigned grid_of(uint64_t n)
{
    const uint64_t g = (n + 255u) / 256u;
    return (unsigned)(g == 0 ? 1u : g);
}

} // namespace

struct nc_gpuhash_mc_parser {
    uint64_t max_bytes, max_reqs, max_keys;
    uint8_t *flag;
    uint64_t *lf;       /* LF positions of complete requests */
    int32_t *status;
    uint32_t *nk;       /* keys per request */
    uint64_t *kbase;    /* exclusive scan of nk */
    uint64_t *kstart;   /* key start in the stream */
    uint32_t *klen;
    uint32_t *kreq;     /* request of each key (when the caller does not want them) */
    uint64_t *misc;     /* [0] selected count, [1] first bad (u64 for atomicMin), [2..] scan totals */
    void *tmp;
    size_t tmp_bytes;
};

static void parser_free(nc_gpuhash_mc_parser_t *ps)
{
    void *bufs[] = {ps->flag, ps->lf, ps->status, ps->nk, ps->kbase, ps->kstart, ps->klen, ps->kreq, ps->misc,
                    ps->tmp};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    free(ps);
}

extern "C" nc_gpuhash_mc_parser_t *nc_gpuhash_mc_parser_create(uint64_t max_bytes, uint64_t max_reqs,
                                                               uint64_t max_keys)
{
    if (max_bytes == 0 || max_reqs == 0 || max_keys == 0 || max_bytes >= (1ull << 31)) {
        errno = EINVAL;
        return nullptr;
    }
    nc_gpuhash_mc_parser_t *ps = (nc_gpuhash_mc_parser_t *)calloc(1, sizeof(*ps));
    if (ps == nullptr) {
        errno = ENOMEM;
        return nullptr;
    }
    ps->max_bytes = max_bytes;
    ps->max_reqs = max_reqs;
    ps->max_keys = max_keys;
    /* temp storage of the largest hipCUB call (select over max_bytes, scans) */
    size_t t1 = 0, t2 = 0, t3 = 0;
    hipError_t e = hipcub::DeviceSelect::Flagged(nullptr, t1, hipcub::CountingInputIterator<uint64_t>(0),
                                                 (uint8_t *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                                 (int64_t)max_bytes);
    if (e == hipSuccess)
        e = hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (uint32_t *)nullptr, (uint64_t *)nullptr, (int64_t)max_reqs + 1);
    if (e == hipSuccess)
        e = hipcub::DeviceScan::ExclusiveSum(nullptr, t3, hipcub::TransformInputIterator<uint64_t, Widen, uint32_t *>(nullptr, Widen()),
                                             (uint64_t *)nullptr, (int64_t)max_keys + 1);
    ps->tmp_bytes = t1 > t2 ? (t1 > t3 ? t1 : t3) : (t2 > t3 ? t2 : t3);
    if (e == hipSuccess) e = hipMalloc((void **)&ps->flag, max_bytes);
    /* the LF select writes every CR LF of the stream before nreq can be
     * checked against max_reqs: size it from the byte limit (one CR LF per
     * two bytes at most), max_reqs only bounds what is reported */
    if (e == hipSuccess) e = hipMalloc((void **)&ps->lf, (max_bytes / 2u + 1u) * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->status, max_reqs * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->nk, (max_reqs + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->kbase, (max_reqs + 1) * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->kstart, max_keys * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->klen, (max_keys + 1) * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->kreq, max_keys * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc((void **)&ps->misc, 8 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&ps->tmp, ps->tmp_bytes ? ps->tmp_bytes : 16u);
    if (e != hipSuccess) {
        parser_free(ps);
        errno = e == hipErrorNoDevice ? ENODEV : ENOMEM;
        return nullptr;
    }
    return ps;
}

extern "C" void nc_gpuhash_mc_parser_destroy(nc_gpuhash_mc_parser_t *ps)
{
    if (ps) parser_free(ps);
}

extern "C" rstatus_t nc_gpuhash_mc_parse_device(nc_gpuhash_mc_parser_t *ps, const uint8_t *d_stream,
                                               uint64_t nbytes, uint8_t *d_keys, uint64_t *d_offsets,
                                               uint32_t *d_key_req, int32_t *d_req_status,
                                               struct nc_gpuhash_mc_result *res, void *stream)
{
    if (ps == nullptr || res == nullptr || (nbytes && d_stream == nullptr) || d_offsets == nullptr) {
        errno = EINVAL;
        return NC_ERROR;
    }
    if (nbytes > ps->max_bytes) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    res->nreqs = res->nkeys = res->consumed = 0;
    res->first_error = 0;
    hipError_t e = hipSuccess;
    uint64_t h[2] = {0, ~0ull};
    if (nbytes) {
        hipLaunchKernelGGL(mc_mark_kernel, dim3(grid_of(nbytes)), dim3(256), 0, st, d_stream, nbytes, ps->flag);
        e = hipGetLastError();
        if (e == hipSuccess)
            e = hipcub::DeviceSelect::Flagged(ps->tmp, ps->tmp_bytes, hipcub::CountingInputIterator<uint64_t>(0),
                                              ps->flag, ps->lf, ps->misc, (int64_t)nbytes, st);
        if (e == hipSuccess) e = hipMemcpyAsync(h, ps->misc, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    const uint64_t nreq = h[0];
    if (e == hipSuccess && nreq > ps->max_reqs) {
        errno = ENOMEM;
        return NC_ENOMEM;
    }
    uint64_t nk = 0, first_bad = nreq;
    if (e == hipSuccess && nreq) {
        e = hipMemcpyAsync(ps->misc + 1, &h[1], sizeof(uint64_t), hipMemcpyHostToDevice, st);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(mc_count_kernel, dim3(grid_of(nreq)), dim3(256), 0, st, d_stream, ps->lf, nreq,
                               ps->status, ps->nk, (unsigned long long *)(ps->misc + 1));
            hipLaunchKernelGGL(mc_clip_kernel, dim3(grid_of(nreq)), dim3(256), 0, st, ps->nk, nreq,
                               (const unsigned long long *)(ps->misc + 1));
            e = hipGetLastError();
        }
        /* nk[nreq] = 0 so the exclusive scan's last element is the key total */
        if (e == hipSuccess) e = hipMemsetAsync(ps->nk + nreq, 0, sizeof(uint32_t), st);
        if (e == hipSuccess)
            e = hipcub::DeviceScan::ExclusiveSum(ps->tmp, ps->tmp_bytes, ps->nk, ps->kbase, (int64_t)nreq + 1, st);
        uint64_t hh[2] = {0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(&hh[0], ps->kbase + nreq, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&hh[1], ps->misc + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        nk = hh[0];
        first_bad = hh[1] < nreq ? hh[1] : nreq;
        if (e == hipSuccess && nk > ps->max_keys) {
            errno = ENOMEM;
            return NC_ENOMEM;
        }
        if (e == hipSuccess && nk) {
            uint32_t *kreq = d_key_req ? d_key_req : ps->kreq;
            hipLaunchKernelGGL(mc_emit_kernel, dim3(grid_of(nreq)), dim3(256), 0, st, d_stream, ps->lf, nreq,
                               (const unsigned long long *)(ps->misc + 1), ps->kbase, ps->kstart, ps->klen, kreq);
            e = hipGetLastError();
            if (e == hipSuccess) e = hipMemsetAsync(ps->klen + nk, 0, sizeof(uint32_t), st);
            hipcub::TransformInputIterator<uint64_t, Widen, uint32_t *> wl(ps->klen, Widen());
            if (e == hipSuccess)
                e = hipcub::DeviceScan::ExclusiveSum(ps->tmp, ps->tmp_bytes, wl, d_offsets, (int64_t)nk + 1, st);
            if (e == hipSuccess && d_keys) {
                hipLaunchKernelGGL(mc_gather_kernel, dim3(grid_of(nk)), dim3(256), 0, st, d_stream, ps->kstart,
                                   d_offsets, nk, d_keys);
                hipLaunchKernelGGL(mc_pad_kernel, dim3(1), dim3(64), 0, st, d_keys, d_offsets, nk);
                e = hipGetLastError();
            }
        }
        if (e == hipSuccess && d_req_status)
            e = hipMemcpyAsync(d_req_status, ps->status, nreq * sizeof(int32_t), hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess && nk == 0) e = hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        errno = e == hipErrorNoDevice ? ENODEV : EIO;
        return NC_ERROR;
    }
    uint64_t consumed = 0;
    if (nreq) {
        /* bytes of the complete requests before the first bad one */
        const uint64_t last = first_bad == 0 ? 0 : first_bad - 1;
        if (first_bad > 0 && hipMemcpy(&consumed, ps->lf + last, sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess)
            consumed += 1;
    }
    res->nreqs = nreq;
    res->nkeys = nk;
    res->first_error = first_bad;
    res->consumed = consumed;
    return NC_OK;
}
