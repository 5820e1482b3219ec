// Calls that may never return, waited for with a deadline.
//
// Some of what the agent reads from sysfs is answered by firmware or hardware, not by the kernel's
// memory: amdgpu's gpu_metrics is an SMU round trip (~1.5 ms per GPU on the box; on an SMU that is
// wedged or resetting the driver waits out its message timeout, per GPU), and a function in PCIe
// error recovery can stall config-space reads (current_link_speed / _width).  The reference bounds
// every wait it has (the 3 s netlink echo, cmd/discover/network.go:242-257; the 5 s pcap read,
// pkg/lldp/client.go:81); these reads get the same treatment.
//
// A Call runs its function on a detached thread, and wait() returns at the deadline whether or
// not the function has.  A call still running is "late": its thread stays blocked in the kernel
// (nothing can cancel a read()), and a new Call under the same key joins it instead of starting
// another, so a wedged device costs one thread, not one per poll.  Unlike std::async's futures,
// nothing here blocks in a destructor.
#pragma once

#include <pthread.h>
#include <time.h>

#include <cerrno>
#include <algorithm>
#include <cstdint>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

namespace netop::bounded {

namespace detail {
// A condition variable on CLOCK_MONOTONIC, waited for with pthread_cond_timedwait.  (libstdc++'s
// steady_clock wait_until goes through pthread_cond_clockwait, which this toolchain's
// ThreadSanitizer does not intercept: every timed wait would read as a double lock.)
class MonoCond {
   public:
    MonoCond() {
        pthread_condattr_t a;
        pthread_condattr_init(&a);
        pthread_condattr_setclock(&a, CLOCK_MONOTONIC);
        pthread_cond_init(&c_, &a);
        pthread_condattr_destroy(&a);
    }
    ~MonoCond() { pthread_cond_destroy(&c_); }
    MonoCond(const MonoCond&) = delete;
    MonoCond& operator=(const MonoCond&) = delete;
    // Waits (lk held) until pred() or CLOCK_MONOTONIC `deadline_ns`; pred()'s value at the end.
    template <class Pred>
    bool wait_until(std::unique_lock<std::mutex>& lk, int64_t deadline_ns, Pred pred) {
        const timespec ts{time_t(deadline_ns / 1000000000), long(deadline_ns % 1000000000)};
        while (!pred())
            if (pthread_cond_timedwait(&c_, lk.mutex()->native_handle(), &ts) == ETIMEDOUT) return pred();
        return true;
    }
    void notify_all() { pthread_cond_broadcast(&c_); }

   private:
    pthread_cond_t c_;
};

struct SlotBase {
    std::mutex m;
    MonoCond cv;
    bool done = false;
    virtual ~SlotBase() = default;
};
// The slot of the call still running under `key`, or `fresh` (then registered under it).  An
// empty key never joins anything.
std::shared_ptr<SlotBase> join_or_register(const std::string& key, const std::shared_ptr<SlotBase>& fresh);
void unregister(const std::string& key, const SlotBase* slot);
// Runs fn on a detached thread; false when no thread could be created.
bool spawn(std::function<void()> fn);
}  // namespace detail

// Calls registered under a key and still running (late ones included).
size_t in_flight();

template <class T>
class Call {
   public:
    Call() = default;
    // Starts fn under `key`, unless a call under that key is still running: then this one is
    // answered by that one.  Without a thread to spare, fn runs in line here.  `notify` (optional)
    // runs on the worker once the result is in place (done() is true by then).
    Call(const std::string& key, std::function<T()> fn, std::function<void()> notify = {}) {
        auto fresh = std::make_shared<Slot>();
        auto s = detail::join_or_register(key, fresh);
        slot_ = std::static_pointer_cast<Slot>(s);
        if (s != fresh) return;
        auto run = [slot = slot_, key, fn = std::move(fn), notify = std::move(notify)] {
            std::optional<T> v;
            std::exception_ptr e;
            try {
                v = fn();
            } catch (...) {
                e = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> g(slot->m);
                slot->value = std::move(v);
                slot->error = e;
                slot->done = true;
            }
            detail::unregister(key, slot.get());
            slot->cv.notify_all();
            if (notify) notify();
        };
        if (!detail::spawn(run)) run();
    }
    bool valid() const { return bool(slot_); }
    // The result, waiting until `deadline_ns` (CLOCK_MONOTONIC, netop::mono_ns()) at most; nullopt
    // when the call has not returned by then.  Rethrows what the function threw.
    std::optional<T> wait(int64_t deadline_ns) const {
        if (!slot_) return std::nullopt;
        std::unique_lock<std::mutex> lk(slot_->m);
        if (!slot_->cv.wait_until(lk, std::max<int64_t>(deadline_ns, 0), [&] { return slot_->done; })) return std::nullopt;
        if (slot_->error) std::rethrow_exception(slot_->error);
        return slot_->value;
    }
    bool done() const {
        if (!slot_) return false;
        std::lock_guard<std::mutex> g(slot_->m);
        return slot_->done;
    }

   private:
    struct Slot : detail::SlotBase {
        std::optional<T> value;
        std::exception_ptr error;
    };
    std::shared_ptr<Slot> slot_;
};

// A file read concurrently with others, each on its own thread, keyed by its path.
struct FileRead {
    std::optional<std::string> data;  // nullopt: unreadable, or late
    bool late = false;                // had not returned by the deadline
};
std::vector<FileRead> read_files(const std::vector<std::string>& paths, int64_t deadline_ns);

}  // namespace netop::bounded
