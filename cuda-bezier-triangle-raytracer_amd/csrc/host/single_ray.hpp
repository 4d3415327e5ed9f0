// single_ray.hpp -- the drop-in's single-ray hot-path methods on the host (single_ray.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>

#include "bzr/bzr.hpp"

namespace bzr {
namespace host {
// BezierTriangle::intersect(ray, limit) (reference/bezierTriangle.cpp:123-195); limitNone = cNone.
BezierIntersection patchIntersect(BezierTriangle const &patch, Ray const &ray, bool limitNone);
// BezierMesh::intersect(ray) (reference/bezierMesh.cpp:206-227); *patch = winning patch, ~0u on a miss.
BezierIntersection meshIntersect(BezierTriangle const *patches, std::size_t n, Ray const &ray, uint32_t *patch);
// BezierLens::refract(ray, expected) (reference/bezierLens.cpp:4-34); the input ray on cNone.
std::pair<Ray, RefractionResult> lensRefract(BezierTriangle const *patches, std::size_t n, float ri, Ray const &ray,
                                             RefractionResult expected);
}  // namespace host
}  // namespace bzr
