// Drop-in forwarding header: the reference file name reference/bezierMesh.h, served by bzr.hpp.
#pragma once
#include "bzr.hpp"
