// Drop-in forwarding header: the reference file name reference/3dGeomUtil.h, served by bzr.hpp.
#pragma once
#include "bzr.hpp"
