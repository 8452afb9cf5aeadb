static const char id[] = "XT_BUILD_ID:f024e0402410c51a44e1d0742914800c";
const char* xt_build_id(void) { return id + 12; }
