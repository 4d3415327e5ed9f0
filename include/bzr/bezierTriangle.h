// Drop-in forwarding header: the reference file name reference/bezierTriangle.h, served by bzr.hpp.
#pragma once
#include "bzr.hpp"
