// Bindings for the BitTorrent / HTTP / storage stack (filled in as those layers land).
#include "bind_extra.h"

void bind_extra(pybind11::module_& m) { (void)m; }
