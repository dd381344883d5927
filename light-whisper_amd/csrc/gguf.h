// Minimal GGUF v3 reader (header, metadata KV, tensor directory; tensor data via mmap).
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace qasr {

enum GgmlType : uint32_t { GGML_F32 = 0, GGML_F16 = 1, GGML_Q8_0 = 8 };

struct GgufValue {
    uint32_t type = 0;            // gguf value type
    int64_t i = 0;
    double f = 0;
    std::string s;
    uint32_t arr_type = 0;
    std::vector<std::string> arr_s;
    std::vector<int64_t> arr_i;
    std::vector<double> arr_f;
};

struct GgufTensor {
    std::string name;
    std::vector<int64_t> dims;   // ggml order: dims[0] = row length
    uint32_t type = 0;
    uint64_t offset = 0;         // relative to data start
    uint64_t nbytes = 0;
    const uint8_t* data = nullptr;
};

class GgufFile {
   public:
    explicit GgufFile(const std::string& path);
    ~GgufFile();
    GgufFile(const GgufFile&) = delete;
    GgufFile& operator=(const GgufFile&) = delete;

    const GgufValue* get(const std::string& key) const;
    int64_t get_int(const std::string& key, int64_t def) const;
    double get_float(const std::string& key, double def) const;
    std::string get_str(const std::string& key, const std::string& def) const;
    const GgufTensor* tensor(const std::string& name) const;
    const std::map<std::string, GgufTensor>& tensors() const { return tensors_; }
    const std::map<std::string, GgufValue>& metadata() const { return kv_; }
    uint32_t version() const { return version_; }

   private:
    std::map<std::string, GgufValue> kv_;
    std::map<std::string, GgufTensor> tensors_;
    uint32_t version_ = 0;
    void* map_ = nullptr;
    size_t size_ = 0;
};

uint64_t ggml_nbytes(uint32_t type, const std::vector<int64_t>& dims);

}  // namespace qasr
