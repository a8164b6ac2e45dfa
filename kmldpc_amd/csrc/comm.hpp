// comm.hpp — RCCL counter all-reduce (comm.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

namespace kml {

constexpr int kCommIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
struct RcclComm;

int rccl_unique_id(unsigned char *out, std::string &err);
// Collective over the world's ranks; the calling thread's current device is the rank's GPU.
RcclComm *rccl_init(const unsigned char *id, int world, int rank, std::string &err);
// In-place sum over the ranks of n uint64 (f64 = false) or double values in device memory, on stream s.
int rccl_allreduce(RcclComm *c, void *buf, size_t n, bool f64, hipStream_t s, std::string &err);
int rccl_size(const RcclComm *c);
void rccl_destroy(RcclComm *c);

}  // namespace kml
