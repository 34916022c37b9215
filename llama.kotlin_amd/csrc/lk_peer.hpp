// lk_peer.hpp — what the chain kernels and their host side (lk_hip.hip, lk_p2p.hip) share.
#pragma once
#include <cstdint>

namespace lk {

constexpr int kChainLine = 32;  // chain sync words: one per 128-B line

// One rank of a multi-GPU chain (lk_p2p_chain): gemv_stream_peer_kernel's view of its peers.
constexpr int kMaxPeerRanks = 8;
struct PeerDesc {
  int32_t P, rank;
  int64_t delta[kMaxPeerRanks];    // byte offset from this rank's dst to rank r's (one layout)
  unsigned *cross[kMaxPeerRanks];  // rank r's cross-rank arrival words, one 128-B line per barrier
  unsigned *epoch;                 // this rank's launch count (a device word)
};

}  // namespace lk
