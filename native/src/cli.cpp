#include "netop/cli.hpp"

#include <stdexcept>

#include "netop/common.hpp"

namespace netop::cli {

static bool parse_bool(const std::string& v, const std::string& flag) {
    if (v == "1" || v == "t" || v == "T" || v == "true" || v == "TRUE" || v == "True") return true;
    if (v == "0" || v == "f" || v == "F" || v == "false" || v == "FALSE" || v == "False") return false;
    throw std::invalid_argument("invalid argument \"" + v + "\" for \"--" + flag + "\" flag: strconv.ParseBool: parsing \"" + v + "\": invalid syntax");
}

void FlagSet::add_string(const std::string& name, std::string* dst, const std::string& help, bool hidden) {
    flags_.push_back({name, help, *dst, false, hidden, [dst](const std::string& v) { *dst = v; }});
}

void FlagSet::add_bool(const std::string& name, bool* dst, const std::string& help, bool hidden) {
    flags_.push_back({name, help, *dst ? "true" : "false", true, hidden,
                      [dst, name](const std::string& v) { *dst = parse_bool(v, name); }});
}

void FlagSet::add_int(const std::string& name, int* dst, const std::string& help, bool hidden) {
    flags_.push_back({name, help, std::to_string(*dst), false, hidden, [dst, name](const std::string& v) {
                          size_t pos = 0;
                          long x = 0;
                          try {
                              x = std::stol(v, &pos, 0);
                          } catch (...) {
                              pos = 0;
                          }
                          if (pos != v.size() || v.empty())
                              throw std::invalid_argument("invalid argument \"" + v + "\" for \"--" + name + "\" flag: parse error");
                          *dst = int(x);
                      }});
}

void FlagSet::add_duration(const std::string& name, int64_t* dst, const std::string& help, bool hidden) {
    flags_.push_back({name, help, format_go_duration(*dst), false, hidden, [dst, name](const std::string& v) {
                          auto d = parse_go_duration(v);
                          if (!d) throw std::invalid_argument("invalid argument \"" + v + "\" for \"--" + name + "\" flag: time: invalid duration \"" + v + "\"");
                          *dst = *d;
                      }});
}

void FlagSet::add_func(const std::string& name, bool takes_value, std::function<void(const std::string&)> fn,
                       const std::string& help, bool hidden) {
    flags_.push_back({name, help, "", !takes_value, hidden, std::move(fn)});
}

void FlagSet::alias(const std::string& a, const std::string& target) { aliases_[a] = target; }
void FlagSet::shorthand(char c, const std::string& target) { shorts_[c] = target; }

FlagSet::Flag* FlagSet::find(const std::string& n) {
    std::string name = n;
    auto a = aliases_.find(name);
    if (a != aliases_.end()) name = a->second;
    for (auto& f : flags_)
        if (f.name == name) return &f;
    return nullptr;
}

std::vector<std::string> FlagSet::parse(int argc, char** argv) {
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--") {
            for (++i; i < argc; ++i) pos.emplace_back(argv[i]);
            break;
        }
        if (a.size() >= 2 && a[0] == '-' && a[1] != '-') {  // shorthand -v 3 / -v=3 / -v3
            char c = a[1];
            auto s = shorts_.find(c);
            if (s == shorts_.end()) throw std::invalid_argument(std::string("unknown shorthand flag: '") + c + "' in " + a);
            Flag* f = find(s->second);
            std::string v;
            if (a.size() > 2)
                v = a[2] == '=' ? a.substr(3) : a.substr(2);
            else if (f->is_bool)
                v = "true";
            else if (i + 1 < argc)
                v = argv[++i];
            else
                throw std::invalid_argument("flag needs an argument: '" + std::string(1, c) + "' in -" + c);
            f->set(v);
            continue;
        }
        if (a.rfind("--", 0) != 0) {
            pos.push_back(a);
            continue;
        }
        std::string body = a.substr(2), name = body, value;
        bool has_value = false;
        auto eq = body.find('=');
        if (eq != std::string::npos) {
            name = body.substr(0, eq);
            value = body.substr(eq + 1);
            has_value = true;
        }
        Flag* f = find(name);
        if (!f) throw std::invalid_argument("unknown flag: --" + name);
        if (!has_value) {
            if (f->is_bool) {
                value = "true";
            } else if (i + 1 < argc) {
                value = argv[++i];
            } else {
                throw std::invalid_argument("flag needs an argument: --" + name);
            }
        }
        f->set(value);
    }
    return pos;
}

std::string FlagSet::usage() const {
    std::string out = "Usage:\n  " + name_ + " [flags]\n\nFlags:\n";
    for (auto& f : flags_) {
        if (f.hidden) continue;
        std::string lhs = "      --" + f.name;
        if (!f.is_bool) lhs += " value";
        if (lhs.size() < 40) lhs.resize(40, ' ');
        out += lhs + " " + f.help;
        if (!f.dflt.empty() && f.dflt != "false") out += " (default " + (f.is_bool ? f.dflt : "\"" + f.dflt + "\"") + ")";
        out += "\n";
    }
    return out;
}

}  // namespace netop::cli
