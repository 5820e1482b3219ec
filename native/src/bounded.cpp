#include "netop/bounded.hpp"

#include <map>
#include <system_error>
#include <thread>

#include "netop/common.hpp"

namespace netop::bounded {

namespace {
std::mutex g_mu;
std::map<std::string, std::shared_ptr<detail::SlotBase>>& registry() {
    static auto* r = new std::map<std::string, std::shared_ptr<detail::SlotBase>>();  // outlives late threads at exit
    return *r;
}
}  // namespace

namespace detail {
std::shared_ptr<SlotBase> join_or_register(const std::string& key, const std::shared_ptr<SlotBase>& fresh) {
    if (key.empty()) return fresh;
    std::lock_guard<std::mutex> g(g_mu);
    auto& r = registry();
    auto it = r.find(key);
    if (it != r.end()) return it->second;
    r.emplace(key, fresh);
    return fresh;
}

void unregister(const std::string& key, const SlotBase* slot) {
    if (key.empty()) return;
    std::lock_guard<std::mutex> g(g_mu);
    auto& r = registry();
    auto it = r.find(key);
    if (it != r.end() && it->second.get() == slot) r.erase(it);
}

bool spawn(std::function<void()> fn) {
    try {
        std::thread(std::move(fn)).detach();
        return true;
    } catch (const std::system_error&) {
        return false;
    }
}
}  // namespace detail

size_t in_flight() {
    std::lock_guard<std::mutex> g(g_mu);
    return registry().size();
}

std::vector<FileRead> read_files(const std::vector<std::string>& paths, int64_t deadline_ns) {
    std::vector<Call<std::optional<std::string>>> calls;
    calls.reserve(paths.size());
    for (const auto& p : paths)  // all started before any is waited for
        calls.emplace_back("file:" + p, [p] { return read_file(p); });
    std::vector<FileRead> out(paths.size());
    for (size_t i = 0; i < calls.size(); ++i) {
        auto r = calls[i].wait(deadline_ns);
        if (!r)
            out[i].late = true;
        else
            out[i].data = std::move(*r);
    }
    return out;
}

}  // namespace netop::bounded
