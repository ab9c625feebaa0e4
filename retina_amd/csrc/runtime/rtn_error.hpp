// Thread-local last-error string shared by every C-ABI entry point of libretina_pc.so
// (rtn_last_error, include/retina_pc.h).
#pragma once
#include <cstdint>
#include <string>

namespace rtn {
int32_t set_error(int32_t code, const std::string& msg);
}
