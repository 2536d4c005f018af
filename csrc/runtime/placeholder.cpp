// Host runtime library (libtfx_rt.so): populated by ps_server.cpp, events.cpp, idx_reader.cpp.
extern "C" int tfx_rt_version() { return 1; }
