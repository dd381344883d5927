#pragma once
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "common.h"
#include "model.h"

namespace qasr {

class Vad {
   public:
    explicit Vad(const std::string& qvad_path);
    ~Vad();
    static int n_frames(int64_t n);
    void features(const float* pcm, int64_t n, std::vector<float>& feats);
    void probabilities(const float* pcm, int64_t n, std::vector<float>& probs);

   private:
    void features_device(const float* pcm, int64_t n, float** d_feats, int* T);
    float* buf(int i, size_t bytes);
    DevAlloc mem_;
    std::map<std::string, float*> arr_;
    float bo_ = 0.f;
    float* win_ = nullptr;
    float* banks_ = nullptr;
    hipStream_t st_ = nullptr;
    std::vector<void*> bufs_;
    std::vector<size_t> caps_;
};

std::vector<std::pair<int64_t, int64_t>> timestamps_from_probabilities(const float* probs, int64_t T,
                                                                       int64_t audio_len, const qasr_vad_options& o);

}  // namespace qasr
