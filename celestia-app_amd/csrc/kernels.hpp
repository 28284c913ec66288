// kernels.hpp -- device kernel launchers shared by the C-ABI layer (dagpu.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dagpu {

constexpr int kShareSize = 512;
constexpr int kNsSize = 29;
constexpr int kNodeSize = 90;  // minNs(29) | maxNs(29) | sha256(32)
constexpr int kDigest = 32;

// Per-square status bits written by the kernels (0 = OK).
constexpr int kStatusPushOrder = 1;

// Generic strided "vector" addressing for the encoder.  For square s, vector v
// and shard i, the input dword column at byte offset `col` lives at
//   in + s*in_sq_stride + v*in_vec_stride + i*in_shard_stride + col.
struct EncodeArgs {
  const uint8_t* in;
  uint8_t* out;
  uint8_t* copy;  // optional: also store the data shards here (Q0 placement)
  long in_sq_stride, in_vec_stride, in_shard_stride;
  long out_sq_stride, out_vec_stride, out_shard_stride;
  long copy_sq_stride, copy_vec_stride, copy_shard_stride;
  long nsq, nvec, nchunk;  // nchunk = ceil(shard_bytes / 512)
  long shard_bytes;
};

hipError_t launch_leo8_encode(int k, const EncodeArgs& a, hipStream_t s);

struct SquareArgs {
  const uint8_t* eds;   // nsq squares, each (2k)^2 * 512 B, row-major
  long eds_sq_stride;
  uint8_t* digests;     // leaf digests: nsq * (2k)^2 * 32 B
  uint8_t* ns_table;    // Q0 namespaces: nsq * k^2 * 32 B
  uint8_t* rec_a;       // tree node records (48 B): nsq * 2w * w/2
  uint8_t* rec_b;       // nsq * 2w * w/4
  uint8_t* row_roots;   // nsq * 2k * 90 B
  uint8_t* col_roots;   // nsq * 2k * 90 B
  uint8_t* dah;         // nsq * 32 B
  int32_t* status;      // nsq status words (kernels OR bits into them)
  int k;
  long nsq;
};

hipError_t launch_nmt_leaves(const SquareArgs& a, hipStream_t s);
// workspace layout for SquareArgs (digests | ns_table | rec_a | rec_b)
size_t nmt_workspace_bytes(int k, long nsq);
void nmt_workspace_carve(SquareArgs& a, void* ws);
hipError_t launch_nmt_trees(const SquareArgs& a, hipStream_t s);
hipError_t launch_dah(const SquareArgs& a, hipStream_t s);

}  // namespace dagpu
