// Internals shared by the C-ABI translation units of libretina_pc.so: the thread-local last-error
// string (rtn_last_error, include/retina_pc.h) and the hiprtc compile cache.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace rtn {
int32_t set_error(int32_t code, const std::string& msg);
// hiprtc-compile a gfx950 code object, cached per process by source hash (rtn_runtime.cpp)
int32_t compile_hip(const std::string& src, std::shared_ptr<std::vector<uint8_t>>& out);
}
