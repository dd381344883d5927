// GGUF v3 reader: parses the header, metadata and tensor directory, mmaps the tensor data (read-only).
#include "gguf.h"

#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "common.h"

namespace qasr {

namespace {
struct Reader {
    const uint8_t* p;
    size_t n, pos = 0;
    template <class T>
    T rd() {
        QASR_CHECK(pos + sizeof(T) <= n, QASR_E_FORMAT, "gguf: truncated file");
        T v;
        memcpy(&v, p + pos, sizeof(T));
        pos += sizeof(T);
        return v;
    }
    std::string str() {
        uint64_t len = rd<uint64_t>();
        QASR_CHECK(len <= n - pos, QASR_E_FORMAT, "gguf: bad string length");
        std::string s((const char*)p + pos, (size_t)len);
        pos += (size_t)len;
        return s;
    }
};

enum : uint32_t {
    GT_U8 = 0, GT_I8, GT_U16, GT_I16, GT_U32, GT_I32, GT_F32, GT_BOOL, GT_STR, GT_ARR, GT_U64, GT_I64, GT_F64
};

void read_scalar(Reader& r, uint32_t t, int64_t& i, double& f, std::string& s) {
    switch (t) {
        case GT_U8: i = r.rd<uint8_t>(); break;
        case GT_I8: i = r.rd<int8_t>(); break;
        case GT_U16: i = r.rd<uint16_t>(); break;
        case GT_I16: i = r.rd<int16_t>(); break;
        case GT_U32: i = r.rd<uint32_t>(); break;
        case GT_I32: i = r.rd<int32_t>(); break;
        case GT_F32: f = r.rd<float>(); i = (int64_t)f; break;
        case GT_BOOL: i = r.rd<uint8_t>(); break;
        case GT_STR: s = r.str(); break;
        case GT_U64: i = (int64_t)r.rd<uint64_t>(); break;
        case GT_I64: i = r.rd<int64_t>(); break;
        case GT_F64: f = r.rd<double>(); i = (int64_t)f; break;
        default: throw Error(QASR_E_FORMAT, "gguf: unknown value type " + std::to_string(t));
    }
    if (t != GT_F32 && t != GT_F64 && t != GT_STR) f = (double)i;
}
}  // namespace

uint64_t ggml_nbytes(uint32_t type, const std::vector<int64_t>& dims) {
    uint64_t n = 1;
    for (auto d : dims) {
        QASR_CHECK(d >= 0 && !__builtin_mul_overflow(n, (uint64_t)d, &n), QASR_E_FORMAT, "gguf: tensor size overflows");
    }
    QASR_CHECK(n <= (UINT64_MAX >> 3), QASR_E_FORMAT, "gguf: tensor size overflows");
    switch (type) {
        case GGML_F32: return n * 4;
        case GGML_F16: return n * 2;
        case GGML_Q8_0:
            QASR_CHECK(!dims.empty() && dims[0] % 32 == 0, QASR_E_FORMAT, "gguf: Q8_0 row not a multiple of 32");
            return n / 32 * 34;
        default: throw Error(QASR_E_FORMAT, "gguf: unsupported tensor type " + std::to_string(type));
    }
}

GgufFile::GgufFile(const std::string& path) {
    int fd = open(path.c_str(), O_RDONLY);
    QASR_CHECK(fd >= 0, QASR_E_IO, "cannot open model file: " + path);
    struct stat st;
    fstat(fd, &st);
    size_ = (size_t)st.st_size;
    map_ = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    QASR_CHECK(map_ != MAP_FAILED, QASR_E_IO, "cannot mmap model file: " + path);
    try {
        Reader r{(const uint8_t*)map_, size_};
        QASR_CHECK(r.rd<uint32_t>() == 0x46554747u, QASR_E_FORMAT, "not a GGUF file: " + path);
        version_ = r.rd<uint32_t>();
        QASR_CHECK(version_ >= 2 && version_ <= 3, QASR_E_FORMAT, "unsupported GGUF version");
        uint64_t n_tensors = r.rd<uint64_t>(), n_kv = r.rd<uint64_t>();
        for (uint64_t k = 0; k < n_kv; k++) {
            std::string key = r.str();
            GgufValue v;
            v.type = r.rd<uint32_t>();
            if (v.type == GT_ARR) {
                v.arr_type = r.rd<uint32_t>();
                uint64_t cnt = r.rd<uint64_t>();
                for (uint64_t j = 0; j < cnt; j++) {
                    int64_t i = 0;
                    double f = 0;
                    std::string s;
                    read_scalar(r, v.arr_type, i, f, s);
                    if (v.arr_type == GT_STR) v.arr_s.push_back(std::move(s));
                    else if (v.arr_type == GT_F32 || v.arr_type == GT_F64) v.arr_f.push_back(f);
                    else v.arr_i.push_back(i);
                }
            } else {
                read_scalar(r, v.type, v.i, v.f, v.s);
            }
            kv_[key] = std::move(v);
        }
        for (uint64_t t = 0; t < n_tensors; t++) {
            GgufTensor ti;
            ti.name = r.str();
            uint32_t nd = r.rd<uint32_t>();
            QASR_CHECK(nd >= 1 && nd <= 4, QASR_E_FORMAT, "gguf: bad tensor rank");
            for (uint32_t d = 0; d < nd; d++) ti.dims.push_back((int64_t)r.rd<uint64_t>());
            ti.type = r.rd<uint32_t>();
            ti.offset = r.rd<uint64_t>();
            ti.nbytes = ggml_nbytes(ti.type, ti.dims);
            tensors_[ti.name] = ti;
        }
        const int64_t align_i = get_int("general.alignment", 32);
        QASR_CHECK(align_i > 0 && align_i <= (1 << 20), QASR_E_FORMAT, "gguf: bad general.alignment");
        const uint64_t align = (uint64_t)align_i;
        const uint64_t data0 = (r.pos + align - 1) / align * align;
        for (auto& kvp : tensors_) {
            auto& ti = kvp.second;
            uint64_t end = 0;
            QASR_CHECK(!__builtin_add_overflow(data0, ti.offset, &end) && !__builtin_add_overflow(end, ti.nbytes, &end) &&
                           end <= size_,
                       QASR_E_FORMAT, "gguf: tensor data out of range: " + ti.name);
            ti.data = (const uint8_t*)map_ + data0 + ti.offset;
        }
    } catch (...) {
        munmap(map_, size_);
        map_ = nullptr;
        throw;
    }
}

GgufFile::~GgufFile() {
    if (map_) munmap(map_, size_);
}

const GgufValue* GgufFile::get(const std::string& key) const {
    auto it = kv_.find(key);
    return it == kv_.end() ? nullptr : &it->second;
}
int64_t GgufFile::get_int(const std::string& key, int64_t def) const {
    auto v = get(key);
    return v && v->type != 8 && v->type != 9 ? v->i : def;
}
double GgufFile::get_float(const std::string& key, double def) const {
    auto v = get(key);
    return v && v->type != 8 && v->type != 9 ? v->f : def;
}
std::string GgufFile::get_str(const std::string& key, const std::string& def) const {
    auto v = get(key);
    return v && v->type == 8 ? v->s : def;
}
const GgufTensor* GgufFile::tensor(const std::string& name) const {
    auto it = tensors_.find(name);
    return it == tensors_.end() ? nullptr : &it->second;
}

}  // namespace qasr
