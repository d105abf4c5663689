// mock_rccl.cpp — TEST INFRASTRUCTURE: an in-process stand-in for the RCCL calls libiblb
// makes (ncclGetUniqueId, ncclCommInitRank, ncclGroupStart/End, ncclSend/Recv,
// ncclAllReduce, ncclAllGather, ncclCommDestroy, ncclGetErrorString), where the ranks are
// host THREADS of one process sharing one GPU.  RCCL itself refuses two ranks on one device,
// so this is how the RCCL slab path of iblb_ctx.hip (peer pairing, message sizes, collective
// order, stream ordering) is exercised on a one-GPU box.  Linked (with -Bsymbolic) into
// tests/mock_rccl/libiblb_mockrccl.so together with the product objects; never shipped.
//
// Semantics kept from RCCL: a send/recv pair matches in posting order per (src, dst); group
// calls post all sends before waiting on any recv; the sender's stream does not run past the
// send until the receiver's copy has finished; collectives are ordered per communicator.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Msg {
    const void* buf = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;
    hipEvent_t copied = nullptr;
    bool done = false;
};

struct World {
    int n = 0;
    int joined = 0;
    std::mutex m;
    std::condition_variable cv;
    std::map<std::pair<int, int>, std::deque<Msg*>> box;
    // generation barrier
    int arrived = 0;
    long gen = 0;
    std::vector<const void*> slot;
};

std::mutex g_m;
std::map<std::string, World*> g_worlds;
std::atomic<long> g_idctr{1};

struct Op {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        default: return 8;
    }
}

void barrier(World* w) {
    std::unique_lock<std::mutex> lk(w->m);
    const long g = w->gen;
    if (++w->arrived == w->n) {
        w->arrived = 0;
        w->gen++;
        w->cv.notify_all();
    } else {
        w->cv.wait(lk, [&] { return w->gen != g; });
    }
}

}  // namespace

struct ncclComm {
    World* w;
    int rank;
};

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error (mock)" : "mock rccl error"; }

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    std::memset(id, 0, sizeof(*id));
    const long k = g_idctr++;
    std::snprintf(id->internal, sizeof(id->internal), "mock-rccl-%ld", k);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    World* w;
    {
        std::lock_guard<std::mutex> lk(g_m);
        std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
        auto it = g_worlds.find(key);
        if (it == g_worlds.end()) {
            w = new World();
            w->n = nranks;
            w->slot.assign(nranks, nullptr);
            g_worlds[key] = w;
        } else {
            w = it->second;
        }
    }
    if (w->n != nranks || rank < 0 || rank >= nranks) return ncclInvalidUsage;
    *comm = new ncclComm{w, rank};
    barrier(w);  // init is collective
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

static ncclResult_t run_group(std::vector<Op>& ops) {
    std::vector<std::pair<Op, Msg*>> sends;
    for (auto& op : ops) {
        if (!op.send) continue;
        Msg* m = new Msg();
        m->buf = op.buf;
        m->bytes = op.bytes;
        if (hipEventCreateWithFlags(&m->ready, hipEventDisableTiming) != hipSuccess) return ncclUnhandledCudaError;
        if (hipEventRecord(m->ready, op.stream) != hipSuccess) return ncclUnhandledCudaError;
        World* w = op.comm->w;
        {
            std::lock_guard<std::mutex> lk(w->m);
            w->box[{op.comm->rank, op.peer}].push_back(m);
        }
        w->cv.notify_all();
        sends.push_back({op, m});
    }
    for (auto& op : ops) {
        if (op.send) continue;
        World* w = op.comm->w;
        Msg* m;
        {
            std::unique_lock<std::mutex> lk(w->m);
            auto& q = w->box[{op.peer, op.comm->rank}];
            w->cv.wait(lk, [&] { return !q.empty(); });
            m = q.front();
            q.pop_front();
        }
        if (m->bytes != op.bytes) return ncclInvalidUsage;  // RCCL would truncate / hang
        if (hipStreamWaitEvent(op.stream, m->ready, 0) != hipSuccess) return ncclUnhandledCudaError;
        if (hipMemcpyAsync(op.buf, m->buf, op.bytes, hipMemcpyDefault, op.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        hipEvent_t cp;
        if (hipEventCreateWithFlags(&cp, hipEventDisableTiming) != hipSuccess) return ncclUnhandledCudaError;
        if (hipEventRecord(cp, op.stream) != hipSuccess) return ncclUnhandledCudaError;
        {
            std::lock_guard<std::mutex> lk(w->m);
            m->copied = cp;
            m->done = true;
        }
        w->cv.notify_all();
    }
    for (auto& sm : sends) {
        World* w = sm.first.comm->w;
        Msg* m = sm.second;
        {
            std::unique_lock<std::mutex> lk(w->m);
            w->cv.wait(lk, [&] { return m->done; });
        }
        // the sender's stream may not overwrite the buffer before the copy finished
        if (hipStreamWaitEvent(sm.first.stream, m->copied, 0) != hipSuccess) return ncclUnhandledCudaError;
        if (hipStreamSynchronize(sm.first.stream) != hipSuccess) return ncclUnhandledCudaError;
        (void)hipEventDestroy(m->ready);
        (void)hipEventDestroy(m->copied);
        delete m;
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    t_depth++;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_group(ops);
}

static ncclResult_t p2p(bool send, const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                        hipStream_t stream) {
    if (!comm || peer < 0 || peer >= comm->w->n) return ncclInvalidArgument;
    Op op{send, const_cast<void*>(buf), count * type_size(dt), peer, comm, stream};
    if (t_depth > 0) {
        t_ops.push_back(op);
        return ncclSuccess;
    }
    std::vector<Op> ops{op};
    return run_group(ops);
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(true, sendbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    return p2p(false, recvbuff, count, datatype, peer, comm, stream);
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
    if (op != ncclSum || (dt != ncclFloat64 && dt != ncclFloat32 && dt != ncclInt32)) return ncclInvalidUsage;
    World* w = comm->w;
    const size_t bytes = count * type_size(dt);
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    w->slot[comm->rank] = sendbuff;
    barrier(w);
    std::vector<char> acc(bytes, 0), tmp(bytes);
    for (int r = 0; r < w->n; ++r) {  // deterministic: rank order
        if (hipMemcpy(tmp.data(), w->slot[r], bytes, hipMemcpyDefault) != hipSuccess) return ncclUnhandledCudaError;
        for (size_t i = 0; i < count; ++i) {
            if (dt == ncclFloat64) ((double*)acc.data())[i] += ((double*)tmp.data())[i];
            else if (dt == ncclFloat32) ((float*)acc.data())[i] += ((float*)tmp.data())[i];
            else ((int*)acc.data())[i] += ((int*)tmp.data())[i];
        }
    }
    barrier(w);  // every rank has read every input before any in-place write
    if (hipMemcpy(recvbuff, acc.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t dt,
                           ncclComm_t comm, hipStream_t stream) {
    World* w = comm->w;
    const size_t bytes = sendcount * type_size(dt);
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    std::vector<char> mine(bytes);
    if (hipMemcpy(mine.data(), sendbuff, bytes, hipMemcpyDefault) != hipSuccess) return ncclUnhandledCudaError;
    w->slot[comm->rank] = mine.data();
    barrier(w);
    std::vector<char> all(bytes * w->n);
    for (int r = 0; r < w->n; ++r) std::memcpy(all.data() + r * bytes, w->slot[r], bytes);
    barrier(w);
    if (hipMemcpy(recvbuff, all.data(), all.size(), hipMemcpyHostToDevice) != hipSuccess) return ncclUnhandledCudaError;
    return ncclSuccess;
}

}  // extern "C"
