static const char id[] = "XT_BUILD_ID:c6b44f5bbeb7630653153089d7bc0238";
const char* xt_build_id(void) { return id + 12; }
