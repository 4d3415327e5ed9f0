// Drop-in for the reference's reference/hostUtil.h: UniformHemisphere (reference/hostUtil.cpp:3-29),
// the emitter's direction sampler.  Header-only and bit-faithful to the reference: the same
// std::ranlux24_base stream and std::uniform_real_distribution<float> draws, and the trig bound as
// the reference binds `::acos(float)` / `::sin` / `::cos` (C's double functions; the products
// `beltRadius * ::cos(turn)` are double, rounded once to float).
//
// The device emitter (bzr_emit / bzr_illuminate, include/bzr.h) samples the same distribution from
// a counter-based stream instead, so any ray range can be generated on any GPU independently.
#pragma once
#include <cmath>
#include <cstdint>
#include <random>
#include <utility>
#include <vector>

#include "3dGeomUtil.h"

class UniformHemisphere final {
private:
  float const cmBeltWidth;
  std::vector<std::pair<float, uint32_t>> mBelts;  // (patch width, first patch index) per belt
  std::ranlux24_base mRandomGenerator;
  std::uniform_real_distribution<float> mUniform1;
  std::uniform_real_distribution<float> mUniform2pi;
  uint32_t mPatchCount;

public:
  explicit UniformHemisphere(uint32_t const aBelts)
      : cmBeltWidth(cgPi / 2.0f / aBelts), mUniform1(0.0f, 1.0f), mUniform2pi(0.0f, cgPi * 2.0f), mPatchCount(0u) {
    mBelts.reserve(aBelts);
    for (uint32_t i = 0u; i < aBelts; ++i) {
      uint32_t now = static_cast<uint32_t>(
          std::ceil(static_cast<double>(4.0f * aBelts) *
                    std::sin(static_cast<double>((2.0f * i + 1.0f) / (4.0f * aBelts) * cgPi))));
      mBelts.emplace_back(cgPi * 2.0f / now, mPatchCount);
      mPatchCount += now;
    }
  }

  uint32_t getPatchCount() const { return mPatchCount; }

  // Unit vector (hemisphere around +x) and its patch index.
  std::pair<Vector, uint32_t> getRandom() {
    Vector direction;
    float incidence = static_cast<float>(std::acos(static_cast<double>(mUniform1(mRandomGenerator))));
    float beltRadius = static_cast<float>(std::sin(static_cast<double>(incidence)));
    auto turn = mUniform2pi(mRandomGenerator);
    direction(0) = static_cast<float>(std::cos(static_cast<double>(incidence)));
    direction(1) = static_cast<float>(beltRadius * std::cos(static_cast<double>(turn)));
    direction(2) = static_cast<float>(beltRadius * std::sin(static_cast<double>(turn)));
    direction.normalize();
    auto const &belt = mBelts[static_cast<uint32_t>(incidence / cmBeltWidth)];
    uint32_t index = belt.second + static_cast<uint32_t>(turn / belt.first);
    return std::pair(direction, index);
  }
};
