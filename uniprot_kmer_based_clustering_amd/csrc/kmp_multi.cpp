// kmp_multi.cpp — transports of the multi-GPU gather (kmp_multi.hpp).
#include "kmp_multi.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdio>

#include "kmerpair.h"

namespace kmp {

namespace {

std::vector<uint64_t> offsets_of(const std::vector<uint64_t>& counts) {
    std::vector<uint64_t> off(counts.size(), 0);
    for (size_t g = 1; g < counts.size(); ++g) off[g] = off[g - 1] + counts[g - 1];
    return off;
}

struct CopyTransport final : Transport {
    std::vector<int> dev;
    explicit CopyTransport(const std::vector<int>& d) : dev(d) {}
    const char* name() const override { return "copy"; }
    int gather(const std::vector<EdgeArrays>& src, const EdgeArrays& dst, const std::vector<uint64_t>& counts,
               const std::vector<hipStream_t>& streams, std::string* err) override {
        const std::vector<uint64_t> off = offsets_of(counts);
        // every copy on rank 0's stream, after every rank's stream drained (the ranks synchronise
        // before the gather anyway: their counts are host values)
        for (size_t g = 0; g < src.size(); ++g) {
            if (!counts[g]) continue;
            for (int a = 0; a < 3; ++a) {
                hipError_t e = hipMemcpyPeerAsync(dst[a] + off[g], dev[0], src[g][a], dev[g], counts[g] * 4, streams[0]);
                if (e != hipSuccess) {
                    *err = std::string("hipMemcpyPeerAsync: ") + hipGetErrorString(e);
                    return KMP_EDEVICE;
                }
            }
        }
        hipError_t e = hipStreamSynchronize(streams[0]);
        if (e != hipSuccess) {
            *err = std::string("gather: ") + hipGetErrorString(e);
            return KMP_EDEVICE;
        }
        return KMP_OK;
    }
    int alltoall(const std::vector<const char*>& send, const std::vector<char*>& recv, uint64_t bytes,
                 const std::vector<hipStream_t>& streams, std::string* err) override {
        const size_t G = send.size();
        for (size_t g = 0; g < G; ++g) {  // every rank's send regions complete
            (void)hipSetDevice(dev[g]);
            hipError_t e = hipStreamSynchronize(streams[g]);
            if (e != hipSuccess) {
                *err = std::string("all-to-all: ") + hipGetErrorString(e);
                return KMP_EDEVICE;
            }
        }
        for (size_t d = 0; d < G; ++d) {
            (void)hipSetDevice(dev[d]);
            for (size_t g = 0; g < G; ++g) {
                hipError_t e = hipMemcpyPeerAsync(recv[d] + g * bytes, dev[d], send[g] + d * bytes, dev[g], bytes,
                                                  streams[d]);
                if (e != hipSuccess) {
                    *err = std::string("hipMemcpyPeerAsync: ") + hipGetErrorString(e);
                    return KMP_EDEVICE;
                }
            }
        }
        for (size_t d = 0; d < G; ++d) {
            (void)hipSetDevice(dev[d]);
            hipError_t e = hipStreamSynchronize(streams[d]);
            if (e != hipSuccess) {
                *err = std::string("all-to-all: ") + hipGetErrorString(e);
                return KMP_EDEVICE;
            }
        }
        (void)hipSetDevice(dev[0]);
        return KMP_OK;
    }
};

// librccl entry points, resolved once per process from /opt/rocm's librccl (RTLD_LOCAL: a
// private instance, independent of any RCCL a host framework loaded)
struct Rccl {
    void* h = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*ErrorString)(ncclResult_t) = nullptr;
    bool load(std::string* err) {
        if (h) return true;
        for (const char* path : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
            h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) {
            *err = std::string("librccl not found: ") + dlerror();
            return false;
        }
        auto sym = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
            return f != nullptr;
        };
        if (!(sym(CommInitAll, "ncclCommInitAll") && sym(CommDestroy, "ncclCommDestroy") && sym(Send, "ncclSend") &&
              sym(Recv, "ncclRecv") && sym(GroupStart, "ncclGroupStart") && sym(GroupEnd, "ncclGroupEnd") &&
              sym(ErrorString, "ncclGetErrorString"))) {
            *err = "librccl lacks an entry point";
            h = nullptr;
            return false;
        }
        return true;
    }
};
Rccl g_rccl;

struct RcclTransport final : Transport {
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    const char* name() const override { return "rccl"; }
    ~RcclTransport() override {
        for (ncclComm_t c : comm)
            if (c) (void)g_rccl.CommDestroy(c);
    }
    int gather(const std::vector<EdgeArrays>& src, const EdgeArrays& dst, const std::vector<uint64_t>& counts,
               const std::vector<hipStream_t>& streams, std::string* err) override {
        const std::vector<uint64_t> off = offsets_of(counts);
        // rank 0's own block: a device copy; the others: one grouped send / receive per array
        for (int a = 0; a < 3 && counts[0]; ++a) {
            hipError_t e = hipMemcpyAsync(dst[a], src[0][a], counts[0] * 4, hipMemcpyDeviceToDevice, streams[0]);
            if (e != hipSuccess) {
                *err = std::string("hipMemcpyAsync: ") + hipGetErrorString(e);
                return KMP_EDEVICE;
            }
        }
        ncclResult_t r = g_rccl.GroupStart();
        for (size_t g = 1; g < src.size() && r == ncclSuccess; ++g) {
            if (!counts[g]) continue;
            for (int a = 0; a < 3 && r == ncclSuccess; ++a) {
                r = g_rccl.Send(src[g][a], counts[g], ncclUint32, 0, comm[g], streams[g]);
                if (r == ncclSuccess) r = g_rccl.Recv(dst[a] + off[g], counts[g], ncclUint32, (int)g, comm[0], streams[0]);
            }
        }
        const ncclResult_t r2 = g_rccl.GroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) {
            *err = std::string("RCCL gather: ") + g_rccl.ErrorString(r);
            return KMP_ERCCL;
        }
        for (size_t g = 0; g < streams.size(); ++g) {
            (void)hipSetDevice(dev[g]);
            hipError_t e = hipStreamSynchronize(streams[g]);
            if (e != hipSuccess) {
                *err = std::string("gather: ") + hipGetErrorString(e);
                return KMP_EDEVICE;
            }
        }
        (void)hipSetDevice(dev[0]);
        return KMP_OK;
    }
    int alltoall(const std::vector<const char*>& send, const std::vector<char*>& recv, uint64_t bytes,
                 const std::vector<hipStream_t>& streams, std::string* err) override {
        const size_t G = send.size();
        // a rank's own region: a device copy; the others: one grouped send / receive per pair,
        // each ordered on its rank's stream after the expansion that filled it
        for (size_t g = 0; g < G; ++g) {
            (void)hipSetDevice(dev[g]);
            hipError_t e = hipMemcpyAsync(recv[g] + g * bytes, send[g] + g * bytes, bytes, hipMemcpyDeviceToDevice,
                                          streams[g]);
            if (e != hipSuccess) {
                *err = std::string("hipMemcpyAsync: ") + hipGetErrorString(e);
                return KMP_EDEVICE;
            }
        }
        ncclResult_t r = g_rccl.GroupStart();
        for (size_t g = 0; g < G && r == ncclSuccess; ++g)
            for (size_t d = 0; d < G && r == ncclSuccess; ++d) {
                if (g == d) continue;
                r = g_rccl.Send(send[g] + d * bytes, bytes / 8, ncclUint64, (int)d, comm[g], streams[g]);
                if (r == ncclSuccess)
                    r = g_rccl.Recv(recv[d] + g * bytes, bytes / 8, ncclUint64, (int)g, comm[d], streams[d]);
            }
        const ncclResult_t r2 = g_rccl.GroupEnd();
        if (r == ncclSuccess) r = r2;
        if (r != ncclSuccess) {
            *err = std::string("RCCL all-to-all: ") + g_rccl.ErrorString(r);
            return KMP_ERCCL;
        }
        for (size_t g = 0; g < G; ++g) {
            (void)hipSetDevice(dev[g]);
            hipError_t e = hipStreamSynchronize(streams[g]);
            if (e != hipSuccess) {
                *err = std::string("all-to-all: ") + hipGetErrorString(e);
                return KMP_EDEVICE;
            }
        }
        (void)hipSetDevice(dev[0]);
        return KMP_OK;
    }
};

}  // namespace

std::unique_ptr<Transport> make_copy_transport(const std::vector<int>& devices) {
    return std::unique_ptr<Transport>(new CopyTransport(devices));
}

std::unique_ptr<Transport> make_rccl_transport(const std::vector<int>& devices, std::string* err) {
    if (!g_rccl.load(err)) return nullptr;
    std::unique_ptr<RcclTransport> t(new RcclTransport);
    t->dev = devices;
    t->comm.assign(devices.size(), nullptr);
    const ncclResult_t r = g_rccl.CommInitAll(t->comm.data(), (int)devices.size(), devices.data());
    if (r != ncclSuccess) {
        *err = std::string("ncclCommInitAll: ") + g_rccl.ErrorString(r);
        t->comm.assign(devices.size(), nullptr);
        return nullptr;
    }
    (void)hipSetDevice(devices[0]);
    return std::unique_ptr<Transport>(t.release());
}

}  // namespace kmp
