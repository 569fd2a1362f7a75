// include/cuZFP.h -- the reference's C++ entry points, served by the MI355X codec.
//
// Same declarations as mclarsen/cuZFP src/cuZFP/cuZFP.h:1-15, so existing
// callers (the reference's gtests, the cuda_zfp CLI) relink unchanged against
// libcuZFP.so.  Semantics follow the reference (cuZFP.cu:174-269):
//   - `field->data` and `stream->stream` may each be host or device memory
//     (detected with hipPointerGetAttributes); host buffers are staged through
//     the device and copied back;
//   - the call is synchronous on the null stream of the current device;
//   - bits per block = stream->maxbits; the stream carries no header;
//   - compress returns the compressed byte count (ceil(blocks*maxbits/64)*8).
// Differences, all in the direction of CPU zfp 0.5.0 (the reference's own
// oracle, src/utils/test.py:68-93): non-zero field strides are honoured; any
// maxbits in [1 + exponent bits, CUZFP_MAX_BITS = 16384] works in every
// dimensionality on gfx950 (zfp's ZFP_MAX_BITS, the most bits a block can use,
// is 4171; on a device with less LDS a block image that does not fit fails
// with CUZFP_ERROR_INVALID_ARGUMENT, include/cuzfp_hip.h);
// partial blocks are padded as CPU zfp pads them; failures print one line to
// stderr and compress returns 0 (the reference prints and continues).
// One addition: cuZFP_last_status() returns the status code (include/cuzfp_hip.h)
// of the calling thread's last compress / decompress, 0 on success, so a caller
// of the void decompress can tell that it failed.
#ifndef cuZFP_h
#define cuZFP_h

#include <stdio.h>

#include <zfp_structs.h>

namespace cuZFP {

size_t compress(zfp_stream* stream, zfp_field* field);
void decompress(zfp_stream* stream, zfp_field* field);

}  // namespace cuZFP

extern "C" int cuZFP_last_status(void);

#endif
