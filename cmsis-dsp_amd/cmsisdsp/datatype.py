"""Datatype tags of the reference's Python binding (PythonWrapper/cmsisdsp_pkg: cmsisdsp.datatype)."""
F64 = 64
F32 = 0
F16 = 3
Q31 = 31
Q15 = 15
Q7 = 7
