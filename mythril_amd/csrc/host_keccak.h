// host_keccak.h — keccak256 of one message on the host (small mq_keccak256 batches).
#pragma once
#include <cstdint>

namespace mq {
void host_keccak256(const uint8_t* msg, int64_t len, uint8_t* out32);
}
