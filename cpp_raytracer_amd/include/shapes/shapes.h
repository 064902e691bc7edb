#ifndef SHAPES_H
#define SHAPES_H

#include "shapes/box.h"
#include "shapes/parallelogram.h"
#include "shapes/sphere.h"

#endif
