import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cmsis-dsp_amd"))
import numpy as np, torch, ctypes as C
import cmsisdsp_amd as dsp
print(dsp.version(), torch.cuda.get_device_name(0))
S = dsp.const_instance("arm_cfft_sR_f32_len1024")
print("fftLen", S.fftLen, "tw", C.cast(S.pTwiddle, C.c_void_p).value, "bitrev", S.bitRevLength)
x = torch.randn(4, 2048, device="cuda")
st = dsp.lib.arm_cfft_f32_batch(C.byref(S), C.c_void_p(x.data_ptr()), 4, 0, 1, C.c_void_p(torch.cuda.current_stream().cuda_stream))
print("status", st, dsp.last_error())
