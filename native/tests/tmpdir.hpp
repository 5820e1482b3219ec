#pragma once

#include <ftw.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string>

#include "netop/common.hpp"

// Self-deleting temporary directory for tests.
struct TmpDir {
    std::string path;
    TmpDir() {
        char tmpl[] = "/tmp/netop-test-XXXXXX";
        char* p = ::mkdtemp(tmpl);
        if (!p) netop::throw_errno("mkdtemp");
        path = p;
    }
    ~TmpDir() {
        ::nftw(path.c_str(), [](const char* f, const struct stat*, int, struct FTW*) { return ::remove(f); }, 16,
               FTW_DEPTH | FTW_PHYS);
    }
    void write(const std::string& rel, const std::string& content) const {
        std::string full = netop::path_join(path, rel);
        netop::mkdir_p(netop::path_dirname(full));
        netop::write_file_atomic(full, content);
    }
    void mkdir(const std::string& rel) const { netop::mkdir_p(netop::path_join(path, rel)); }
    void symlink(const std::string& target_rel, const std::string& link_rel) const {
        std::string link = netop::path_join(path, link_rel);
        netop::mkdir_p(netop::path_dirname(link));
        if (::symlink(netop::path_join(path, target_rel).c_str(), link.c_str()) != 0) netop::throw_errno("symlink " + link);
    }
};
