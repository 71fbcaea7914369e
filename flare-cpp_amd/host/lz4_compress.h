// lz4_compress.h -- a CompressHandler for COMPRESS_TYPE_LZ4
// (/root/reference/flare/rpc/options.proto:74), shaped like the Snappy one
// (/root/reference/flare/rpc/policy/snappy_compress.h:30-42: same four
// functions, same meaning of arguments and return values).  The reference
// registers nothing at this type; GlobalInitializeLz4() is the registration a
// maintainer would add beside global.cc:372-376.
//
// Per call the host codec runs (host/lz4_cpu.h): one body is one serial LZ4
// walk, which a CPU core runs faster than one GPU lane.  The GPU LZ4 kernels
// serve batches through include/flare_lz4_gpu.h.
#pragma once

#include "compress.h"
#include "cord_buf.h"

namespace flare::rpc::policy {

bool Lz4Compress(const Message& msg, cord_buf* buf);
bool Lz4Decompress(const cord_buf& data, Message* msg);
bool Lz4Compress(const cord_buf& in, cord_buf* out);
bool Lz4Decompress(const cord_buf& in, cord_buf* out);

}  // namespace flare::rpc::policy

namespace flare::rpc {
// Registers the LZ4 handler at COMPRESS_TYPE_LZ4 once per process; 0 on
// success.
int GlobalInitializeLz4();
}  // namespace flare::rpc
