// Drop-in forwarding header: the reference file name reference/mesh.h, served by bzr.hpp.
#pragma once
#include "bzr.hpp"
