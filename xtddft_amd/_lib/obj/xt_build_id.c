static const char id[] = "XT_BUILD_ID:a21fb5f85ca3b3cf17bd0ed0d2367112";
const char* xt_build_id(void) { return id + 12; }
