extern "C" const char* gpi_source_sha(void) { return "921dc086b6a93a0ab6694d0b10cd3b2106015a40"; }
