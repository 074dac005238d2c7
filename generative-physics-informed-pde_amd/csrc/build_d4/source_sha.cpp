extern "C" const char* gpi_source_sha(void) { return "a07d060b410a01c68daa9de4159f317d66ecfafd"; }
