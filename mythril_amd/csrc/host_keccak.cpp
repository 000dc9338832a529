// host_keccak.cpp — keccak256 (Ethereum padding 0x01..0x80, rate 136 B) on the host, for the
// small batches of mq_keccak256: find_concrete_keccak (keccak_function_manager.py:56-69) and
// _replace_with_actual_sha (analysis/solver.py:131-167) hash one to a few messages per call, and a
// GPU launch plus two copies (~50 us) costs more than hashing them here (~1 us per 136-byte block).
// keccak-f[1600] on 64-bit lanes, rho offsets and pi permutation folded into one table walk.
#include <cstdint>
#include <cstring>

#include "host_keccak.h"

namespace mq {
namespace {

constexpr uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// the pi walk: lane kPiLane[i] receives the previous lane rotated by kRho[i] (starting at lane 1)
constexpr int kPiLane[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
constexpr int kRho[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};

inline uint64_t rotl(uint64_t v, int n) { return (v << n) | (v >> (64 - n)); }

void keccak_f1600(uint64_t (&a)[25]) {
  for (int r = 0; r < 24; r++) {
    uint64_t c[5];
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
      for (int y = 0; y < 25; y += 5) a[y + x] ^= d;
    }
    uint64_t t = a[1];
    for (int i = 0; i < 24; i++) {
      const int j = kPiLane[i];
      const uint64_t u = a[j];
      a[j] = rotl(t, kRho[i]);
      t = u;
    }
    for (int y = 0; y < 25; y += 5) {
      uint64_t row[5];
      for (int x = 0; x < 5; x++) row[x] = a[y + x];
      for (int x = 0; x < 5; x++) a[y + x] = row[x] ^ (~row[(x + 1) % 5] & row[(x + 2) % 5]);
    }
    a[0] ^= kRC[r];
  }
}

inline uint64_t load_le64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);   // (x86-64 and the GPU box's hosts are little-endian)
  return v;
}

}  // namespace

void host_keccak256(const uint8_t* msg, int64_t len, uint8_t* out32) {
  uint64_t a[25] = {};
  int64_t pos = 0;
  for (; len - pos >= 136; pos += 136) {
    for (int w = 0; w < 17; w++) a[w] ^= load_le64(msg + pos + 8 * w);
    keccak_f1600(a);
  }
  uint8_t last[136] = {};
  std::memcpy(last, msg + pos, (size_t)(len - pos));
  last[len - pos] ^= 0x01;
  last[135] ^= 0x80;
  for (int w = 0; w < 17; w++) a[w] ^= load_le64(last + 8 * w);
  keccak_f1600(a);
  std::memcpy(out32, a, 32);
}

}  // namespace mq
