// options.h -- process-wide tuning and test options of libflare_snappy_gpu.so.
//
// Each option starts from its FSG_<NAME> environment variable, read ONCE when
// the library is loaded (A/B tooling sets them per process), and is changed
// afterwards only through fsg_set_option (include/flare_snappy_gpu.h).  The
// launch paths read the table's atomics, never the environment: getenv is not
// safe against a concurrent setenv in a multi-threaded server, and a variable
// must not silently change what a running process launches.
#pragma once
#include <cstdint>

namespace fsg {

enum Opt : int {
  // Snappy two-pass decode (snappy_decode_v4.hip)
  kOptDecodeFork,         // -1 automatic (> 128K messages), 0 one stream, 1 forked path
  kOptSplitWalk,          // forked small-message execution order 0..3 (3 default)
  kOptSplitClass,         // walk class split point of mode 3
  kOptExecKeep,           // history kept at a window slide (bytes, 512..kMaxKeep, multiple of 16)
  kOptChunkedHuge,        // chunked pass 1b for the huge bodies of the forked path
  kOptSmallPersist,       // forked small-message grid (blocks; 0 = a wave per message)
  kOptSmallBatch,         // batches of at most this many messages index on pass 1b
  kOptSplitHuge,          // huge bodies on a second side stream
  kOptWalkOrder,          // planned lane walk in size-class order
  kOptLeanWalk,           // two-stream form: the lean lane walk
  kOptExecBigBlocks,      // one-stream exec launch: large-message blocks
  kOptExecPrio,           // exec pass priority raise around round-A loads
  kOptExecBigBlocksFork,  // forked path: large-message exec blocks
  kOptExecPack,           // forked path: short bodies per packed execution batch (0 = a wave per body)
  // Snappy encode (capi.hip, snappy_encode_v3.hip)
  kOptEncodeWaveMin,      // long-unit threshold of the wave encoder (bytes; 0 = lanes only)
  kOptEncodeWaveShare,    // wave encoder's share of long units (permille)
  kOptEncodeWaveAllMb,    // all long units to the wave encoder below this many MiB
  kOptEncodeLanes,        // lanes in flight of the lane encoder (0 = all)
  kOptEncodeWavePerCu,    // wave encoder waves per CU (0 = as many as LDS holds)
  kOptEncodeWaveWg,       // wave encoder waves per workgroup (1..5; their tables share the workgroup's LDS)
  // LZ4 two-pass decode (lz4_decode2.hip)
  kOptLz4BigMin,          // -1 automatic; blocks above this many bytes take the wave walk
  kOptCount
};

// Current value (relaxed load).
int64_t opt(Opt o);

}  // namespace fsg
