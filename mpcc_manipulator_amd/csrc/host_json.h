// host_json.h — minimal JSON reader for the Params/*.json and track files (host only).
// Supports objects, arrays, numbers, strings, true/false/null — what nlohmann::json is used for in
// the reference's loaders (params.cpp, track.cpp).  Throws std::runtime_error on malformed input;
// the C-ABI layer converts that into MPCC_E_IO.
#pragma once
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace mpcc {

struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    double num = 0;
    bool b = false;
    std::string str;
    std::vector<JVal> arr;
    std::map<std::string, JVal> obj;

    bool has(const std::string& k) const { return kind == OBJ && obj.count(k); }
    const JVal& at(const std::string& k) const {
        auto it = obj.find(k);
        if (kind != OBJ || it == obj.end()) throw std::runtime_error("json: missing key '" + k + "'");
        return it->second;
    }
    double number() const {
        if (kind == NUM) return num;
        if (kind == BOOL) return b ? 1.0 : 0.0;
        throw std::runtime_error("json: value is not a number");
    }
    std::vector<double> numbers() const {
        if (kind != ARR) throw std::runtime_error("json: value is not an array");
        std::vector<double> v;
        v.reserve(arr.size());
        for (auto& e : arr) v.push_back(e.number());
        return v;
    }
};

class JParser {
   public:
    explicit JParser(const std::string& s) : s_(s) {}
    JVal parse() {
        JVal v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

   private:
    const std::string& s_;
    size_t i_ = 0;
    [[noreturn]] void fail(const char* m) {
        throw std::runtime_error(std::string("json parse error: ") + m + " at offset " + std::to_string(i_));
    }
    void ws() {
        while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) i_++;
    }
    JVal value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        if (c == '{') return object();
        if (c == '[') return array();
        if (c == '"') { JVal v; v.kind = JVal::STR; v.str = string(); return v; }
        if (s_.compare(i_, 4, "true") == 0) { i_ += 4; JVal v; v.kind = JVal::BOOL; v.b = true; return v; }
        if (s_.compare(i_, 5, "false") == 0) { i_ += 5; JVal v; v.kind = JVal::BOOL; v.b = false; return v; }
        if (s_.compare(i_, 4, "null") == 0) { i_ += 4; return JVal(); }
        return number();
    }
    JVal number() {
        const char* b = s_.c_str() + i_;
        char* e = nullptr;
        double d = std::strtod(b, &e);  // correctly rounded, as nlohmann::json
        if (e == b) fail("bad number");
        i_ += (size_t)(e - b);
        JVal v;
        v.kind = JVal::NUM;
        v.num = d;
        return v;
    }
    std::string string() {
        if (s_[i_] != '"') fail("expected string");
        i_++;
        std::string out;
        while (i_ < s_.size() && s_[i_] != '"') {
            if (s_[i_] == '\\') {
                i_++;
                if (i_ >= s_.size()) fail("bad escape");
                char e = s_[i_];
                out += (e == 'n') ? '\n' : (e == 't') ? '\t' : e;
            } else {
                out += s_[i_];
            }
            i_++;
        }
        if (i_ >= s_.size()) fail("unterminated string");
        i_++;
        return out;
    }
    JVal array() {
        JVal v;
        v.kind = JVal::ARR;
        i_++;
        ws();
        if (i_ < s_.size() && s_[i_] == ']') { i_++; return v; }
        for (;;) {
            v.arr.push_back(value());
            ws();
            if (i_ >= s_.size()) fail("unterminated array");
            if (s_[i_] == ',') { i_++; continue; }
            if (s_[i_] == ']') { i_++; return v; }
            fail("expected , or ]");
        }
    }
    JVal object() {
        JVal v;
        v.kind = JVal::OBJ;
        i_++;
        ws();
        if (i_ < s_.size() && s_[i_] == '}') { i_++; return v; }
        for (;;) {
            ws();
            std::string k = string();
            ws();
            if (i_ >= s_.size() || s_[i_] != ':') fail("expected :");
            i_++;
            v.obj[k] = value();
            ws();
            if (i_ >= s_.size()) fail("unterminated object");
            if (s_[i_] == ',') { i_++; continue; }
            if (s_[i_] == '}') { i_++; return v; }
            fail("expected , or }");
        }
    }
};

inline JVal json_load_file(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    std::string s = ss.str();
    JParser p(s);
    return p.parse();
}

}  // namespace mpcc
