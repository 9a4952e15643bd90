// Declaration-only stand-in for the reference's common/logger.hpp (spdlog logger): see
// ../boss_chunk_construct.hpp.
#pragma once
#include <memory>
#include <string>

namespace mtg::common {
struct Logger {
    template <typename... Args>
    void error(const char *fmt, Args &&...args);
};
extern std::shared_ptr<Logger> logger;
}  // namespace mtg::common
