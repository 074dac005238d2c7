extern "C" const char* gpi_source_sha(void) { return "d1a42813cd3668ef7d9434fdb821976f2a690eaf"; }
