// comm.cpp -- the aggregation step across GPUs as a C ABI over RCCL.
//
// The reference merges per-partition aggregator state with RDD.treeAggregate
// (core/src/main/scala/org/apache/spark/rdd/RDD.scala:1210-1269: seqOp per
// partition, foldByKey tree levels :1244-1250, driver fold :1267), KMeans'
// reduceByKey + collectAsMap (mllib/clustering/KMeans.scala:308-311) and a
// DoubleAccumulator, and ships the model with TorrentBroadcast
// (SparkContext.scala:1524).  With one executor process per GPU, each
// process owns one communicator and replaces all of that with ONE in-place
// fp64 sum of its flat state buffer per iteration (ncclAllReduce over xGMI)
// plus a broadcast of the model -- callable from a JVM shim without Python
// (INTEGRATION.md).  The 128-byte unique id travels out of band (the Spark
// driver's broadcast, a torch.distributed store, a file).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "common.hpp"

struct cyc_comm_s {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
  std::mutex mu;                // host-pointer calls share the staging buffer
  hipStream_t st = nullptr;     // stream of the host-pointer calls
  cyc::DeviceBuffer stage;
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
  cyc::set_error(std::string("RCCL error in ") + what + ": " + ncclGetErrorString(r));
  return CYC_ERR_HIP;
}

#define CYC_NCCL(expr)                                      \
  do {                                                      \
    ncclResult_t _r = (expr);                               \
    if (_r != ncclSuccess) return nccl_fail(_r, #expr);     \
  } while (0)

int check_comm(cyc_comm c) {
  CYC_REQUIRE(c != nullptr && c->comm != nullptr, "communicator must not be null");
  return CYC_OK;
}

// RCCL counts are size_t; every fp64 buffer of the path (<= 8 MB, SURVEY
// 8(e)) is far below any limit, so only the sign is checked.
int check_count(int64_t count) {
  CYC_REQUIRE(count >= 0, "count must be nonnegative but got " + std::to_string(count));
  return CYC_OK;
}

}  // namespace

extern "C" {

int cyc_comm_unique_id(unsigned char* id) {
  CYC_REQUIRE(id != nullptr, "id must not be null");
  ncclUniqueId u;
  CYC_NCCL(ncclGetUniqueId(&u));
  static_assert(sizeof(u.internal) == CYC_COMM_ID_BYTES, "unique id size");
  std::memcpy(id, u.internal, CYC_COMM_ID_BYTES);
  return CYC_OK;
}

int cyc_comm_init(const unsigned char* id, int32_t rank, int32_t world, int32_t device,
                  cyc_comm* out) {
  CYC_REQUIRE(id != nullptr && out != nullptr, "id and out must not be null");
  CYC_REQUIRE(world >= 1, "world size must be positive but got " + std::to_string(world));
  CYC_REQUIRE(rank >= 0 && rank < world,
              "rank must be in [0, " + std::to_string(world) + ") but got " +
                  std::to_string(rank));
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    cyc::set_error("no HIP device visible");
    return CYC_ERR_NO_DEVICE;
  }
  CYC_REQUIRE(device >= 0 && device < ndev,
              "device must be in [0, " + std::to_string(ndev) + ") but got " +
                  std::to_string(device));
  CYC_HIP(hipSetDevice(device));
  ncclUniqueId u;
  std::memcpy(u.internal, id, CYC_COMM_ID_BYTES);
  auto* c = new cyc_comm_s();
  c->rank = rank;
  c->world = world;
  c->device = device;
  ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) {
    (void)ncclCommDestroy(c->comm);
    delete c;
    cyc::set_error("hipStreamCreateWithFlags failed");
    return CYC_ERR_HIP;
  }
  *out = c;
  return CYC_OK;
}

int cyc_comm_destroy(cyc_comm c) {
  if (!c) return CYC_OK;
  int rc = CYC_OK;
  if (c->st) {
    (void)hipStreamSynchronize(c->st);
    (void)hipStreamDestroy(c->st);
  }
  if (c->comm) {
    ncclResult_t r = ncclCommDestroy(c->comm);
    if (r != ncclSuccess) rc = nccl_fail(r, "ncclCommDestroy");
  }
  delete c;
  return rc;
}

int cyc_comm_rank(cyc_comm c, int32_t* rank, int32_t* world) {
  if (int rc = check_comm(c)) return rc;
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  return CYC_OK;
}

int cyc_allreduce_sum_dev(cyc_comm c, double* buf, int64_t count, void* stream) {
  if (int rc = check_comm(c)) return rc;
  if (int rc = check_count(count)) return rc;
  if (count == 0) return CYC_OK;
  CYC_REQUIRE(buf != nullptr, "buffer must not be null");
  CYC_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, c->comm,
                         cyc::as_stream(stream)));
  return CYC_OK;
}

int cyc_allreduce_max_dev(cyc_comm c, double* buf, int64_t count, void* stream) {
  if (int rc = check_comm(c)) return rc;
  if (int rc = check_count(count)) return rc;
  if (count == 0) return CYC_OK;
  CYC_REQUIRE(buf != nullptr, "buffer must not be null");
  CYC_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclMax, c->comm,
                         cyc::as_stream(stream)));
  return CYC_OK;
}

int cyc_broadcast_dev(cyc_comm c, double* buf, int64_t count, int32_t root, void* stream) {
  if (int rc = check_comm(c)) return rc;
  if (int rc = check_count(count)) return rc;
  CYC_REQUIRE(root >= 0 && root < c->world, "root must be a rank of the communicator");
  if (count == 0) return CYC_OK;
  CYC_REQUIRE(buf != nullptr, "buffer must not be null");
  CYC_NCCL(ncclBroadcast(buf, buf, (size_t)count, ncclFloat64, root, c->comm,
                         cyc::as_stream(stream)));
  return CYC_OK;
}

int cyc_allgather_dev(cyc_comm c, const double* send, double* recv, int64_t count,
                      void* stream) {
  if (int rc = check_comm(c)) return rc;
  if (int rc = check_count(count)) return rc;
  if (count == 0) return CYC_OK;
  CYC_REQUIRE(send != nullptr && recv != nullptr, "buffers must not be null");
  CYC_NCCL(ncclAllGather(send, recv, (size_t)count, ncclFloat64, c->comm,
                         cyc::as_stream(stream)));
  return CYC_OK;
}

// Host-pointer forms for the resident-dataset layer (its outputs are host
// arrays): staged through a device buffer on the communicator's stream,
// synchronous.
int cyc_allreduce_sum(cyc_comm c, double* host_buf, int64_t count) {
  if (int rc = check_comm(c)) return rc;
  if (int rc = check_count(count)) return rc;
  if (count == 0) return CYC_OK;
  CYC_REQUIRE(host_buf != nullptr, "buffer must not be null");
  std::lock_guard<std::mutex> g(c->mu);
  CYC_HIP(hipSetDevice(c->device));
  const size_t bytes = sizeof(double) * (size_t)count;
  if (int rc = c->stage.reserve(bytes)) return rc;
  CYC_HIP(hipMemcpyAsync(c->stage.ptr, host_buf, bytes, hipMemcpyHostToDevice, c->st));
  CYC_NCCL(ncclAllReduce(c->stage.ptr, c->stage.ptr, (size_t)count, ncclFloat64, ncclSum,
                         c->comm, c->st));
  CYC_HIP(hipMemcpyAsync(host_buf, c->stage.ptr, bytes, hipMemcpyDeviceToHost, c->st));
  CYC_HIP(hipStreamSynchronize(c->st));
  return CYC_OK;
}

int cyc_broadcast(cyc_comm c, double* host_buf, int64_t count, int32_t root) {
  if (int rc = check_comm(c)) return rc;
  if (int rc = check_count(count)) return rc;
  CYC_REQUIRE(root >= 0 && root < c->world, "root must be a rank of the communicator");
  if (count == 0) return CYC_OK;
  CYC_REQUIRE(host_buf != nullptr, "buffer must not be null");
  std::lock_guard<std::mutex> g(c->mu);
  CYC_HIP(hipSetDevice(c->device));
  const size_t bytes = sizeof(double) * (size_t)count;
  if (int rc = c->stage.reserve(bytes)) return rc;
  if (c->rank == root)
    CYC_HIP(hipMemcpyAsync(c->stage.ptr, host_buf, bytes, hipMemcpyHostToDevice, c->st));
  CYC_NCCL(ncclBroadcast(c->stage.ptr, c->stage.ptr, (size_t)count, ncclFloat64, root, c->comm,
                         c->st));
  CYC_HIP(hipMemcpyAsync(host_buf, c->stage.ptr, bytes, hipMemcpyDeviceToHost, c->st));
  CYC_HIP(hipStreamSynchronize(c->st));
  return CYC_OK;
}

}  // extern "C"
