// Tiny pflag-compatible command-line parser (--name=value, --name value, -v N, bool
// flags with optional =true/false), used by the agent binaries.  The reference uses
// cobra + pflag + klog's Go flag set (cmd/discover/main.go:263-301).
#pragma once

#include <functional>
#include <map>
#include <string>
#include <vector>

namespace netop::cli {

class FlagSet {
   public:
    explicit FlagSet(std::string name) : name_(std::move(name)) {}
    void add_string(const std::string& name, std::string* dst, const std::string& help, bool hidden = false);
    void add_bool(const std::string& name, bool* dst, const std::string& help, bool hidden = false);
    void add_int(const std::string& name, int* dst, const std::string& help, bool hidden = false);
    void add_duration(const std::string& name, int64_t* dst_ns, const std::string& help, bool hidden = false);
    void add_func(const std::string& name, bool takes_value, std::function<void(const std::string&)> fn,
                  const std::string& help, bool hidden = false);
    void alias(const std::string& alias, const std::string& target);
    void shorthand(char c, const std::string& target);

    // Throws std::invalid_argument with a pflag-like message.  Returns positional args.
    std::vector<std::string> parse(int argc, char** argv);
    std::string usage() const;

   private:
    struct Flag {
        std::string name, help, dflt;
        bool is_bool = false;
        bool hidden = false;
        std::function<void(const std::string&)> set;
    };
    Flag* find(const std::string& n);
    std::string name_;
    std::vector<Flag> flags_;
    std::map<std::string, std::string> aliases_;
    std::map<char, std::string> shorts_;
};

}  // namespace netop::cli
