#include <cstdio>
#include <cstring>

#include "check.hpp"
#include "netop/log.hpp"

namespace netop_test {
std::vector<Case>& registry() {
    static std::vector<Case> r;
    return r;
}
}  // namespace netop_test

int main(int argc, char** argv) {
    // Keep the agent's logging out of the test report unless asked for.
    static std::string sink;
    bool verbose = false;
    const char* filter = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "-v"))
            verbose = true;
        else
            filter = argv[i];
    }
    if (!verbose) netop::log::set_capture(&sink);
    int failed = 0, ran = 0;
    for (auto& c : netop_test::registry()) {
        if (filter && !std::strstr(c.name, filter)) continue;
        std::fprintf(stderr, "RUN  %s\n", c.name);
        ++ran;
        try {
            c.fn();
            std::printf("PASS %s\n", c.name);
            std::fflush(stdout);
        } catch (const std::exception& e) {
            ++failed;
            std::printf("FAIL %s: %s\n", c.name, e.what());
        }
        sink.clear();
    }
    std::printf("%d/%d passed\n", ran - failed, ran);
    return failed ? 1 : 0;
}
