// gguf_reader.h -- GGUF v3 parser over a caller-owned byte buffer.
//
// Behaviour follows the reference loader (gguf.cpp:158-304): little-endian
// header {magic, version, n_tensors, n_kv}, typed metadata values (arrays
// recursive), tensor infos {name, n_dims, dims[], type, offset}, tensor data
// section at the next 32-byte boundary (general.alignment ignored, as in the
// reference).  Errors throw gguf_error with the reference's messages.
#pragma once

#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace llmi {

struct gguf_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct GValue {
  uint32_t type = 4;  // GGUFType (gguf.h:14-28)
  double num = 0;     // numeric scalars widened
  uint32_t u32 = 0;   // raw low 32 bits (the reference reads scalar.u32 / .f32)
  std::string str;
  std::vector<GValue> arr;
  float f32() const { float f; std::memcpy(&f, &u32, 4); return f; }
};

struct GTensor {
  std::string name;
  std::vector<uint64_t> shape;
  uint32_t type = 0;
  uint64_t offset = 0;
};

class GGUFView {
 public:
  GGUFView(const uint8_t* data, size_t size) : p_(data), n_(size) { load(); }

  const std::map<std::string, GValue>& metadata() const { return meta_; }
  const std::vector<GTensor>& tensors() const { return tensors_; }
  const uint8_t* tensor_data(const GTensor& t) const { return p_ + data_start_ + t.offset; }
  size_t size() const { return n_; }
  size_t data_start() const { return data_start_; }

  const GValue* find(const std::string& k) const {
    auto it = meta_.find(k);
    return it == meta_.end() ? nullptr : &it->second;
  }
  const GTensor* tensor(const std::string& name) const {
    for (const auto& t : tensors_)
      if (t.name == name) return &t;
    return nullptr;
  }

 private:
  const uint8_t* p_;
  size_t n_, pos_ = 0, data_start_ = 0;
  std::map<std::string, GValue> meta_;
  std::vector<GTensor> tensors_;

  template <typename T>
  T rd() {
    if (pos_ + sizeof(T) > n_) throw gguf_error("Read beyond end of file");
    T v;
    std::memcpy(&v, p_ + pos_, sizeof(T));
    pos_ += sizeof(T);
    return v;
  }
  std::string rd_str() {
    const uint64_t len = rd<uint64_t>();
    if (len > n_) throw gguf_error("Invalid string length: " + std::to_string(len));
    if (pos_ + len > n_) throw gguf_error("String length exceeds file size");
    std::string s(reinterpret_cast<const char*>(p_ + pos_), len);
    pos_ += len;
    return s;
  }
  GValue rd_value(uint32_t type) {
    GValue v;
    v.type = type;
    auto scalar = [&](auto x) {
      v.num = (double)x;
      uint64_t raw = 0;
      std::memcpy(&raw, &x, sizeof(x));
      v.u32 = (uint32_t)raw;
    };
    switch (type) {
      case 0: scalar(rd<uint8_t>()); break;
      case 1: scalar(rd<int8_t>()); break;
      case 2: scalar(rd<uint16_t>()); break;
      case 3: scalar(rd<int16_t>()); break;
      case 4: scalar(rd<uint32_t>()); break;
      case 5: scalar(rd<int32_t>()); break;
      case 6: scalar(rd<float>()); break;
      case 7: scalar(rd<uint8_t>()); break;
      case 8: v.str = rd_str(); break;
      case 9: {
        const uint32_t et = rd<uint32_t>();
        const uint64_t cnt = rd<uint64_t>();
        v.num = (double)cnt;
        v.arr.reserve(cnt < (1u << 24) ? cnt : 0);
        for (uint64_t i = 0; i < cnt; i++) v.arr.push_back(rd_value(et));
        break;
      }
      case 10: scalar(rd<uint64_t>()); break;
      case 11: scalar(rd<int64_t>()); break;
      case 12: scalar(rd<double>()); break;
      default: throw gguf_error("Unsupported GGUF value type");
    }
    return v;
  }
  void load() {
    if (rd<uint32_t>() != 0x46554747u) throw gguf_error("Invalid GGUF magic number");
    rd<uint32_t>();  // version
    const uint64_t nt = rd<uint64_t>(), nkv = rd<uint64_t>();
    for (uint64_t i = 0; i < nkv; i++) {
      std::string k = rd_str();
      const uint32_t t = rd<uint32_t>();
      meta_[k] = rd_value(t);
    }
    for (uint64_t i = 0; i < nt; i++) {
      GTensor t;
      t.name = rd_str();
      const uint32_t nd = rd<uint32_t>();
      for (uint32_t d = 0; d < nd; d++) t.shape.push_back(rd<uint64_t>());
      t.type = rd<uint32_t>();
      t.offset = rd<uint64_t>();
      tensors_.push_back(std::move(t));
    }
    data_start_ = (pos_ + 31) & ~size_t(31);
  }
};

}  // namespace llmi
