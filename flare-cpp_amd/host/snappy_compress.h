// snappy_compress.h -- the snappy CompressHandler, GPU-backed.
// Same names, argument meaning and return values as
// /root/reference/flare/rpc/policy/snappy_compress.h:30-42.
#pragma once

#include "compress.h"
#include "cord_buf.h"

namespace flare::rpc::policy {

// Compress serialized `msg' into `buf' (appended).
bool SnappyCompress(const Message& msg, cord_buf* buf);

// Parse `msg' from decompressed `data'.
bool SnappyDecompress(const cord_buf& data, Message* msg);

// Put compressed `in' into `out' (appended).
bool SnappyCompress(const cord_buf& in, cord_buf* out);

// Put decompressed `in' into `out' (appended).
bool SnappyDecompress(const cord_buf& in, cord_buf* out);

}  // namespace flare::rpc::policy

namespace flare::rpc {
// Registers the GPU snappy handler at COMPRESS_TYPE_SNAPPY once per process,
// as GlobalInitializeOrDieImpl does (/root/reference/flare/rpc/global.cc:372-376).
// Returns 0 on success (or if already registered by this call earlier).
int GlobalInitializeSnappyGpu();
}  // namespace flare::rpc
