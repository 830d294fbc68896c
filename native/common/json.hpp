// Minimal JSON value, parser and pretty-printer for the native tools (sdk-cli, sdk-bootstrap).
// Objects keep insertion order so printed output matches what the scheduler sent.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace sdk {

class Json {
 public:
  enum class Type { Null, Bool, Number, String, Array, Object };
  using Array = std::vector<Json>;
  using Object = std::vector<std::pair<std::string, Json>>;

  Json() : type_(Type::Null) {}
  Json(std::nullptr_t) : type_(Type::Null) {}
  Json(bool b) : type_(Type::Bool), b_(b) {}
  Json(double d) : type_(Type::Number), n_(d) {}
  Json(int i) : type_(Type::Number), n_(i) {}
  Json(const char* s) : type_(Type::String), s_(s) {}
  Json(std::string s) : type_(Type::String), s_(std::move(s)) {}
  static Json array() {
    Json j;
    j.type_ = Type::Array;
    j.a_ = std::make_shared<Array>();
    return j;
  }
  static Json object() {
    Json j;
    j.type_ = Type::Object;
    j.o_ = std::make_shared<Object>();
    return j;
  }

  Type type() const { return type_; }
  bool is_null() const { return type_ == Type::Null; }
  bool is_string() const { return type_ == Type::String; }
  bool is_array() const { return type_ == Type::Array; }
  bool is_object() const { return type_ == Type::Object; }
  bool is_number() const { return type_ == Type::Number; }
  bool is_bool() const { return type_ == Type::Bool; }

  const std::string& str() const;
  double num() const;
  bool boolean() const;
  const Array& arr() const;
  Array& arr();
  const Object& obj() const;

  // object access: returns a null Json when absent
  const Json& operator[](const std::string& key) const;
  bool has(const std::string& key) const;
  void set(const std::string& key, Json v);
  void push(Json v);
  size_t size() const;

  static Json parse(const std::string& text);
  std::string dump(int indent = -1) const;
  // a string value as-is, anything else as compact JSON
  std::string as_text() const { return is_string() ? s_ : dump(); }

 private:
  void dump_to(std::string& out, int indent, int level) const;
  Type type_;
  bool b_ = false;
  double n_ = 0;
  std::string s_;
  std::shared_ptr<Array> a_;
  std::shared_ptr<Object> o_;
};

class JsonError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

}  // namespace sdk
