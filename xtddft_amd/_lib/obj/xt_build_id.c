static const char id[] = "XT_BUILD_ID:fc005ff7614c737b4068ab3aa11c8b7d";
const char* xt_build_id(void) { return id + 12; }
