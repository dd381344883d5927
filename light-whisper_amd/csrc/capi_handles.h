// The opaque handles of include/qasr.h (shared by the extern "C" translation units).
#pragma once
#include <memory>

#include "engine.h"
#include "vad.h"

struct qasr_model {
    std::unique_ptr<qasr::Model> m;
};
struct qasr_session {
    std::unique_ptr<qasr::Session> s;
};
struct qasr_vad {
    std::unique_ptr<qasr::Vad> v;
};
