// Minimal HTTP/1.1 endpoint for the node agent: GET /metrics (Prometheus text exposition),
// /healthz and /readyz.  One background thread, blocking accept, one request per connection,
// 2 s socket timeouts — it serves scrapes, nothing else.  The agent publishes pre-rendered
// documents with set_*(); the server never calls back into the agent (no locking of agent
// state from another thread).
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

namespace netop::httpd {

class Server {
   public:
    // addr: "host:port" or ":port" (port 0 = ephemeral).  Throws SysError on bind failure.
    explicit Server(const std::string& addr);
    ~Server();
    Server(const Server&) = delete;
    Server& operator=(const Server&) = delete;

    int port() const { return port_; }
    void set_metrics(std::string text);
    void set_ready(bool ready) { ready_ = ready; }
    uint64_t requests() const { return requests_; }

   private:
    void loop();
    void handle(int fd);

    int fd_ = -1;
    int port_ = 0;
    std::atomic<bool> stop_{false};
    std::atomic<bool> ready_{false};
    std::atomic<uint64_t> requests_{0};
    std::mutex mu_;
    std::string metrics_;
    std::thread th_;
};

// Prometheus text helpers.
std::string escape_label(const std::string& v);

}  // namespace netop::httpd
