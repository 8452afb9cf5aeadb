static const char id[] = "XT_BUILD_ID:90c8e26bb25cc6f2aa2600046cee66c8";
const char* xt_build_id(void) { return id + 12; }
