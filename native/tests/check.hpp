// Minimal self-registering unit-test harness (no gtest in this image).
#pragma once

#include <functional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace netop_test {

struct Case {
    const char* name;
    std::function<void()> fn;
};
std::vector<Case>& registry();
struct Reg {
    Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
struct Failure : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <class A, class B>
void check_eq(const A& a, const B& b, const char* ea, const char* eb, const char* file, int line) {
    if (!(a == b)) {
        std::ostringstream os;
        os << file << ":" << line << ": CHECK_EQ(" << ea << ", " << eb << ") failed: [" << a << "] != [" << b << "]";
        throw Failure(os.str());
    }
}

}  // namespace netop_test

#define NT_CAT2(a, b) a##b
#define NT_CAT(a, b) NT_CAT2(a, b)
#define TEST(name)                                                  \
    static void name();                                             \
    static ::netop_test::Reg NT_CAT(reg_, name)(#name, name);      \
    static void name()

#define CHECK(cond)                                                                                              \
    do {                                                                                                         \
        if (!(cond)) throw ::netop_test::Failure(std::string(__FILE__) + ":" + std::to_string(__LINE__) + ": CHECK(" #cond ") failed"); \
    } while (0)

#define CHECK_EQ(a, b) ::netop_test::check_eq((a), (b), #a, #b, __FILE__, __LINE__)

#define CHECK_THROWS(expr)                                                                                        \
    do {                                                                                                          \
        bool thrown_ = false;                                                                                     \
        try {                                                                                                     \
            (void)(expr);                                                                                         \
        } catch (...) {                                                                                           \
            thrown_ = true;                                                                                       \
        }                                                                                                         \
        if (!thrown_) throw ::netop_test::Failure(std::string(__FILE__) + ":" + std::to_string(__LINE__) + ": expected exception from " #expr); \
    } while (0)
