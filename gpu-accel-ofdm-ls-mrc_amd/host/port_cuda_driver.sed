# port_cuda_driver.sed -- the mechanical edits that turn the reference's CUDA
# driver (gpuLS_main.cu) into a HIP driver against host/gpuLS.hpp:
#   sed -f port_cuda_driver.sed gpuLS_main.cu > gpuLS_main.cpp
# 1. the class header and the CUDA library headers
s/#include "gpuLS.cuh"/#include "gpuLS.hpp"/
/#include <cufft.h>/d
/#include <cublas_v2.h>/d
/#include <cuComplex.h>/d
/#include "cuda_runtime.h"/d
/#include "device_launch_parameters.h"/d
/#include <cuda_profiler_api.h>/d
# 2. the cuFFT warm-up plan (no plans here: the library's FFT has none)
/^[[:space:]]*cufft/d
# 3. CUDA type and runtime names -> HIP
s/cuFloatComplex/hipFloatComplex/g
s/cudaSetDevice/hipSetDevice/g
s/cudaMalloc/hipMalloc/g
s/cudaMemcpy/hipMemcpy/g
s/cudaFree/hipFree/g
s/cudaDeviceSynchronize/hipDeviceSynchronize/g
s/cudaStream_t/hipStream_t/g
# 4. gpuLS_main.cu:104,107,112 call gpuLS methods as free functions, which
#    does not compile as published: call them on one gpuLS object, created
#    right after the device is selected (its constructor attaches to the ring)
/hipSetDevice(0);/a\
	gpuLS gpu;
s/^\([[:space:]]*\)copyPilotToGPU(/\1gpu.copyPilotToGPU(/
s/^\([[:space:]]*\)firstVector(/\1gpu.firstVector(/
s/^\([[:space:]]*\)demodOneSymbol(/\1gpu.demodOneSymbol(/
