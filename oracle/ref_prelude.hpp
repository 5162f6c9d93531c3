/*
 * ref_prelude.hpp -- force-included in front of the reference functions that
 * oracle/build_ref.sh extracts from /root/reference/cpuLS.hpp.
 *
 * TEST INFRASTRUCTURE ONLY.  It supplies nothing the image lacks: complexF and
 * the config macros come from the reference's own ShMemSymBuff.hpp (found via
 * -I/root/reference); the only local definition is the pilot-file name that
 * cpuLS.hpp:41 hard-codes, made a variable so tests can point it at a fixture.
 */
#include "ShMemSymBuff.hpp"
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
using namespace std;
static const char *g_ref_pilot_path = "Pilots.dat";
#define fileNameForX g_ref_pilot_path
