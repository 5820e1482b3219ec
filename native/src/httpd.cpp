#include "netop/httpd.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstring>

#include "netop/common.hpp"
#include "netop/log.hpp"

namespace netop::httpd {

std::string escape_label(const std::string& v) {
    std::string o;
    for (char c : v) {
        if (c == '\\' || c == '"') o += '\\';
        if (c == '\n') {
            o += "\\n";
            continue;
        }
        o += c;
    }
    return o;
}

Server::Server(const std::string& addr) {
    auto colon = addr.rfind(':');
    std::string host = colon == std::string::npos ? "" : addr.substr(0, colon);
    int port = std::stoi(colon == std::string::npos ? addr : addr.substr(colon + 1));
    fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd_ < 0) throw_errno("socket(metrics)");
    int one = 1;
    ::setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(uint16_t(port));
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (!host.empty() && host != "0.0.0.0" && ::inet_pton(AF_INET, host.c_str(), &sa.sin_addr) != 1) {
        ::close(fd_);
        throw SysError(EINVAL, "metrics address " + addr);
    }
    if (::bind(fd_, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 || ::listen(fd_, 16) != 0) {
        int e = errno;
        ::close(fd_);
        throw SysError(e, "bind metrics " + addr);
    }
    socklen_t sl = sizeof sa;
    ::getsockname(fd_, reinterpret_cast<sockaddr*>(&sa), &sl);
    port_ = ntohs(sa.sin_port);
    th_ = std::thread([this] { loop(); });
}

Server::~Server() {
    stop_ = true;
    if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
    if (th_.joinable()) th_.join();
    if (fd_ >= 0) ::close(fd_);
}

void Server::set_metrics(std::string text) {
    std::lock_guard<std::mutex> lk(mu_);
    metrics_ = std::move(text);
}

void Server::loop() {
    while (!stop_) {
        pollfd p{fd_, POLLIN, 0};
        int r = ::poll(&p, 1, 200);
        if (r <= 0) continue;
        int c = ::accept4(fd_, nullptr, nullptr, SOCK_CLOEXEC);
        if (c < 0) continue;
        timeval tv{2, 0};
        ::setsockopt(c, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
        ::setsockopt(c, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
        handle(c);
        ::close(c);
    }
}

void Server::handle(int c) {
    char buf[2048];
    size_t got = 0;
    while (got < sizeof buf - 1) {
        ssize_t n = ::recv(c, buf + got, sizeof buf - 1 - got, 0);
        if (n <= 0) return;
        got += size_t(n);
        buf[got] = 0;
        if (std::strstr(buf, "\r\n\r\n") || std::strstr(buf, "\n\n")) break;
    }
    ++requests_;
    std::string req(buf, got);
    auto sp1 = req.find(' '), sp2 = req.find(' ', sp1 + 1);
    std::string method = req.substr(0, sp1), path = sp1 == std::string::npos ? "" : req.substr(sp1 + 1, sp2 - sp1 - 1);
    int code = 200;
    std::string body, type = "text/plain; charset=utf-8";
    if (method != "GET") {
        code = 405;
        body = "method not allowed\n";
    } else if (path == "/metrics") {
        std::lock_guard<std::mutex> lk(mu_);
        body = metrics_;
        type = "text/plain; version=0.0.4; charset=utf-8";
    } else if (path == "/healthz") {
        body = "ok\n";
    } else if (path == "/readyz") {
        code = ready_ ? 200 : 503;
        body = ready_ ? "ok\n" : "not ready\n";
    } else {
        code = 404;
        body = "not found\n";
    }
    const char* reason = code == 200 ? "OK" : code == 404 ? "Not Found" : code == 405 ? "Method Not Allowed" : "Service Unavailable";
    std::string resp = strfmt("HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %zu\r\nConnection: close\r\n\r\n", code,
                              reason, type.c_str(), body.size()) +
                       body;
    size_t off = 0;
    while (off < resp.size()) {
        ssize_t n = ::send(c, resp.data() + off, resp.size() - off, MSG_NOSIGNAL);
        if (n <= 0) return;
        off += size_t(n);
    }
}

}  // namespace netop::httpd
