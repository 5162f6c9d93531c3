// ShMemSymBuff_gpu.hpp -- drop-in for the reference's ShMemSymBuff_gpu.hpp: the shared-memory
// symbol ring (ShMemSymBuff_impl.hpp) with this header's default geometry
// (ShMemSymBuff_gpu.hpp:48-80): numOfRows 16, lenOfBuffer 101, dimension 1024, prefix 0, each
// overridable with -D.  Like the reference's three ring headers it uses the
// include guard _SHMEMSYMBUFF_HPP_, so the first ring header a translation
// unit includes fixes the geometry and the others are no-ops.
#ifndef _SHMEMSYMBUFF_HPP_
#define _SHMEMSYMBUFF_HPP_

#ifndef numOfRows
#define numOfRows 16
#endif
#ifndef lenOfBuffer
#define lenOfBuffer 101
#endif

#include "ShMemSymBuff_impl.hpp"

#endif  // _SHMEMSYMBUFF_HPP_
