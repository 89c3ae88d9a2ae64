// json.h -- the JSON report writer of the host tool.
//
// The reference writes its report with the vendored nlohmann::json 3.5.0 `dump(4)`
// (reference src/jsonreporter.cpp:160, src/json.hpp): objects keyed through std::map (bytewise
// sorted keys), 4-space indentation, one array element per line, integers verbatim and doubles
// through Grisu2 (src/json.hpp:9761-10819).  This is an independent implementation of that
// output format so that reports are byte-identical.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace fqhost {

// Shortest-ish round-trip decimal for a double exactly as the reference's JSON writer prints it
// (Grisu2 digits, %g-like layout with fixed notation for 1e-5 < |v| < 1e15, "null" for NaN/Inf).
std::string json_double(double v);

class Json {
   public:
    enum Kind { Null, Int, UInt, Double, String, Array, Object };
    Json() : kind_(Null) {}
    static Json i(int64_t v) { Json j; j.kind_ = Int; j.i_ = v; return j; }
    static Json u(uint64_t v) { Json j; j.kind_ = UInt; j.u_ = v; return j; }
    static Json d(double v) { Json j; j.kind_ = Double; j.d_ = v; return j; }
    static Json s(const std::string& v) { Json j; j.kind_ = String; j.s_ = v; return j; }
    static Json array() { Json j; j.kind_ = Array; return j; }
    static Json object() { Json j; j.kind_ = Object; return j; }
    // object member access (creates an object from null, like nlohmann's operator[])
    Json& operator[](const std::string& key);
    void push(const Json& v);
    Kind kind() const { return kind_; }
    std::string dump(int indent) const;

   private:
    void dump_to(std::string& out, int indent, int level) const;
    Kind kind_;
    int64_t i_ = 0;
    uint64_t u_ = 0;
    double d_ = 0;
    std::string s_;
    std::vector<Json> arr_;
    std::map<std::string, Json> obj_;
};

}  // namespace fqhost
