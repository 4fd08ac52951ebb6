// json_config.hpp -- the reader LoopHandler's constructor needs (src/LoopHandler.cc:8-16: Json::Reader::parse of
// config/KITTI*.json, then value["basePath"].asString() etc.).  jsoncpp is not in this image, so this parses the
// subset those files use: one top-level object of string / number / bool / null members, with jsoncpp's default
// comment support (// and /* */, as in config/KITTI_mock_test.json).  A missing key reads as "" (asString() of a
// null Json::Value).  Nested objects and arrays are skipped over, not kept.
#pragma once

#include <cctype>
#include <fstream>
#include <map>
#include <sstream>
#include <string>

namespace yavo_fe {

class JsonConfig {
public:
    bool parse(const std::string& text) {
        s_ = text;
        i_ = 0;
        values_.clear();
        ws();
        if (!eat('{')) return false;
        ws();
        if (eat('}')) return true;
        while (true) {
            ws();
            std::string key;
            if (!str(key)) return false;
            ws();
            if (!eat(':')) return false;
            ws();
            std::string val;
            if (!value(val)) return false;
            values_[key] = val;
            ws();
            if (eat(',')) continue;
            return eat('}');
        }
    }
    bool parse_file(const std::string& path) {
        std::ifstream f(path);
        if (!f) return false;
        std::stringstream ss;
        ss << f.rdbuf();
        return parse(ss.str());
    }
    // Json::Value::asString(): strings as written, numbers / bools as their text, missing -> ""
    std::string asString(const std::string& key) const {
        auto it = values_.find(key);
        return it == values_.end() ? std::string() : it->second;
    }
    bool has(const std::string& key) const { return values_.count(key) != 0; }

private:
    std::string s_;
    size_t i_ = 0;
    std::map<std::string, std::string> values_;

    bool eat(char c) {
        if (i_ < s_.size() && s_[i_] == c) {
            ++i_;
            return true;
        }
        return false;
    }
    void ws() {
        while (i_ < s_.size()) {
            if (std::isspace((unsigned char)s_[i_])) {
                ++i_;
            } else if (s_.compare(i_, 2, "//") == 0) {
                while (i_ < s_.size() && s_[i_] != '\n') ++i_;
            } else if (s_.compare(i_, 2, "/*") == 0) {
                const size_t e = s_.find("*/", i_ + 2);
                i_ = e == std::string::npos ? s_.size() : e + 2;
            } else {
                break;
            }
        }
    }
    bool str(std::string& out) {
        if (!eat('"')) return false;
        out.clear();
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\' && i_ < s_.size()) {
                const char e = s_[i_++];
                switch (e) {
                    case 'n': c = '\n'; break;
                    case 't': c = '\t'; break;
                    case 'r': c = '\r'; break;
                    case 'b': c = '\b'; break;
                    case 'f': c = '\f'; break;
                    default: c = e; break;  // \" \\ \/ (\u escapes are not used by the configs)
                }
            }
            out.push_back(c);
        }
        return eat('"');
    }
    bool skip_nested(char open, char close) {
        int depth = 0;
        while (i_ < s_.size()) {
            const char c = s_[i_];
            if (c == '"') {
                std::string tmp;
                if (!str(tmp)) return false;
                continue;
            }
            ++i_;
            if (c == open) ++depth;
            if (c == close && --depth == 0) return true;
        }
        return false;
    }
    bool value(std::string& out) {
        if (i_ >= s_.size()) return false;
        const char c = s_[i_];
        if (c == '"') return str(out);
        if (c == '{') { out.clear(); return skip_nested('{', '}'); }
        if (c == '[') { out.clear(); return skip_nested('[', ']'); }
        const size_t b = i_;
        while (i_ < s_.size() && !std::isspace((unsigned char)s_[i_]) && s_[i_] != ',' && s_[i_] != '}' &&
               s_.compare(i_, 2, "//") != 0 && s_.compare(i_, 2, "/*") != 0)
            ++i_;
        out = s_.substr(b, i_ - b);
        if (out == "null") out.clear();
        return !out.empty() || s_.compare(b, 4, "null") == 0;
    }
};

}  // namespace yavo_fe
