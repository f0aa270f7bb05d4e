// Additional pybind11 registrations for the host core, split across translation units.
#pragma once
#include <pybind11/pybind11.h>

void bind_extra(pybind11::module_& m);
