// Communication backend: replaces the reference's El::mpi collective overload
// sets and their Aluminum/NCCL glue (src/core/imports/mpi/{AllGather,ReduceScatter,
// AllToAll,SendRecv,Broadcast}.hpp, include/El/core/imports/aluminum.hpp:24-365).
//
//   * RCCL (device buffers): one communicator per grid dimension, built with
//     ncclCommSplit from the world communicator; collectives are enqueued on the
//     caller's HIP stream (never host-blocking, unlike the reference's plain-MPI
//     path which calls hipStreamSynchronize before every collective,
//     src/core/imports/mpi/AllGather.hpp:36).  Irregular exchanges are grouped
//     ncclSend/ncclRecv: on xGMI every peer pair has its own link, so a direct
//     exchange uses c-1 links at once instead of one ring neighbour.
//   * HOST (host buffers): the caller supplies the collective as a callback
//     (e.g. torch.distributed/gloo); device buffers are staged through pinned
//     host memory.  Used by the CPU multi-rank tests.
//   * SELF: size-1 communicator, every collective is a local copy.
#pragma once
#include "../common.hpp"
#include "../runtime/runtime.hpp"
#include <memory>
#include <vector>
#include <rccl/rccl.h>

namespace elx {

struct CommStats {
    int64_t bytes = 0;   // algorithmic bytes received by this rank
    int64_t calls = 0;
    double seconds = 0;  // host wall time spent inside host-backend collectives
};
CommStats& GlobalCommStats();

// Transfer-only timing of device collectives (HIP events on the stream the
// RCCL group runs on; pack/unpack launches excluded): the xGMI GB/s figure.
struct CommProfiler {
    struct Rec { hipEvent_t a = nullptr, b = nullptr; int64_t bytes = 0; };
    bool on = false;
    std::vector<Rec> recs;
    void Clear();
    Rec Begin(hipStream_t s);
    void End(Rec r, hipStream_t s, int64_t bytes);
    // summed transfer ms, bytes received, number of timed transfers
    void Stats(double& ms, int64_t& bytes, int64_t& calls);
};
CommProfiler& CommProf();

// Stage watchdog (replaces the fencing the reference gets from MPI's and
// Aluminum's own error handling, include/El/core/imports/mpi/aluminum_comm.hpp:174-212):
// a background thread that ends the process with exit code kWatchdogExit,
// naming the stage on stderr, when the armed stage overruns its deadline or an
// owned RCCL communicator reports an asynchronous error.  Every live owned RCCL
// communicator is aborted first (ncclCommAbort) so no GPU kernel is left
// spinning on a peer.  seconds <= 0 keeps the stage name but disarms the deadline.
constexpr int kWatchdogExit = 75;
void WatchdogStage(const char* name, double seconds);
// text written to stdout when the watchdog fires (empty: nothing), and the exit
// status it then uses (kWatchdogExit until set)
void WatchdogEpitaph(const char* text, int exit_code);
void WatchdogRegister(ncclComm_t c);
void WatchdogUnregister(ncclComm_t c);

// One-to-all byte broadcast over TCP (rank 0 serves `addr:port`): the RCCL
// unique-id exchange MPI_Bcast does for the reference's Aluminum init, for
// processes started by torch.distributed.run (RANK / WORLD_SIZE / MASTER_ADDR).
void RendezvousBcast(void* data, size_t bytes, int rank, int size, const char* addr, int port, double timeout_s);


// El::mpi::Op for the reductions (include/El/core/imports/mpi.hpp:88-99): the
// ops an RCCL reduction supports natively
enum class ReduceOp : int { SUM = ELX_OP_SUM, PROD = ELX_OP_PROD, MAX = ELX_OP_MAX, MIN = ELX_OP_MIN };

class Comm {
public:
    enum class Kind { SELF, RCCL, HOST };

    static std::shared_ptr<Comm> Self();
    static std::shared_ptr<Comm> InitRCCL(int rank, int size, const unsigned char id[128]);
    // borrow a caller's RCCL communicator (never destroyed here); splits of it are owned
    static std::shared_ptr<Comm> WrapRCCL(ncclComm_t c);
    static std::shared_ptr<Comm> InitHost(int rank, int size, elx_host_coll_fn coll, elx_host_split_fn split,
                                          void* ctx);
    ~Comm();

    Kind kind() const { return kind_; }
    int Rank() const { return rank_; }
    int Size() const { return size_; }
    // Collective over this comm: ranks with equal color form a new comm ordered by key.
    std::shared_ptr<Comm> Split(int color, int key);

    // All counts are in elements of `t`; `dev` says where the buffers live.
    void AllGather(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s);
    void ReduceScatter(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s,
                       ReduceOp op = ReduceOp::SUM);
    void AllReduce(DType t, const void* send, void* recv, Int count, Device dev, hipStream_t s,
                   ReduceOp op = ReduceOp::SUM);
    void Bcast(DType t, void* buf, Int count, int root, Device dev, hipStream_t s);
    // Irregular all-to-all: sendcounts/recvcounts per peer (elements), with
    // element displacements into send/recv.  Pairs with zero count are skipped.
    void AllToAllV(DType t, const void* send, const std::vector<Int>& scounts, const std::vector<Int>& sdispls,
                   void* recv, const std::vector<Int>& rcounts, const std::vector<Int>& rdispls, Device dev,
                   hipStream_t s);
    // Several AllToAllV exchanges of one communicator in ONE RCCL group (every
    // set's sends and receives posted together, so exchanges with disjoint peer
    // sets use their links concurrently); the host backend carries them in one
    // all-to-all with the same per-peer set order (ELX_GROUPED_EXCHANGE=0: the
    // sets run as separate exchanges on either backend).
    struct VSet {
        DType t;
        const void* send;
        const std::vector<Int>* sc;
        const std::vector<Int>* sd;
        void* recv;
        const std::vector<Int>* rc;
        const std::vector<Int>* rd;
    };
    void AllToAllVGroup(const std::vector<VSet>& sets, Device dev, hipStream_t s);
    // Point-to-point exchange (El::mpi::SendRecv, src/core/imports/mpi/SendRecv.hpp:9-60):
    // send `count` elements to `dest` while receiving `count` from `src`.
    void SendRecv(DType t, const void* send, int dest, void* recv, int src, Int count, Device dev, hipStream_t s);
    // separate send / receive counts (SendRecv.hpp:9-35's sc / rc); the host
    // backend's callback carries one count, so there they must be equal
    void SendRecv(DType t, const void* send, Int scount, int dest, void* recv, Int rcount, int src, Device dev,
                  hipStream_t s);
    void Barrier();

private:
    Comm() = default;
    void HostCall(int op, DType t, const void* send, void* recv, Int count, int peer, int peer2);
    void HostGroup(const std::vector<VSet>& sets, Device dev, hipStream_t s);
    // Host-backend reductions the callback does not do itself (16-bit sums, the
    // reference's own MPI_Op, src/core/environment.cpp:135-142,259-298; every
    // non-SUM op): gather the contributions and fold them in rank order
    void HostFold(bool scatter, DType t, ReduceOp op, const void* send, void* recv, Int count, Device dev,
                  hipStream_t s);
    Kind kind_ = Kind::SELF;
    int rank_ = 0, size_ = 1;
    ncclComm_t nccl_ = nullptr;
    bool owned_ = true;
    elx_host_coll_fn coll_ = nullptr;
    elx_host_split_fn split_ = nullptr;
    void* ctx_ = nullptr;
    int group_ = 0;
};

// The world communicator El::mpi::COMM_WORLD resolves to (size 1 until one is
// installed); InitWorldFromEnv builds an RCCL world from the launcher's env.
std::shared_ptr<Comm>& WorldComm();
void InitWorldFromEnv();

}  // namespace elx
