// ShMemSymBuff_cucomplex.hpp -- drop-in for the reference's ShMemSymBuff_cucomplex.hpp: the shared-memory
// symbol ring (ShMemSymBuff_impl.hpp) with this header's default geometry
// (ShMemSymBuff_cucomplex.hpp:48-83): numOfRows 1, lenOfBuffer 117, dimension 1024, prefix 0, each
// overridable with -D.  Like the reference's three ring headers it uses the
// include guard _SHMEMSYMBUFF_HPP_, so the first ring header a translation
// unit includes fixes the geometry and the others are no-ops.
#ifndef _SHMEMSYMBUFF_HPP_
#define _SHMEMSYMBUFF_HPP_

#ifndef numOfRows
#define numOfRows 1
#endif
#ifndef lenOfBuffer
#define lenOfBuffer 117
#endif

#include "ShMemSymBuff_impl.hpp"

#endif  // _SHMEMSYMBUFF_HPP_
