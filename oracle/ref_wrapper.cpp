// ref_wrapper.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Emulates what the reference's clang JIT does to a plugin source before
// compiling it: the plugin file is included verbatim and three extern "C"
// entry points are appended (ref compiler.cpp:1181-1203, and the setjmp
// error wrapper of wrapper_plugin_object.cpp:102-115).  The plugin source
// itself is read from its place under /root/reference; nothing is copied.
//
// Build: see oracle/Makefile (REF_PLUGIN_SRC = path of the plugin .cpp).

#include REF_PLUGIN_SRC

extern "C" void audio_callback_type_wrapper(void *param_ptr, void *state_ptr,
                                            float **out_buffer,
                                            unsigned int num_channels,
                                            unsigned int num_samples,
                                            float sample_rate)
{
    audio_callback(*(Parameters *)param_ptr, *(State *)state_ptr, out_buffer,
                   num_channels, num_samples, sample_rate);
}

extern "C" void default_parameters_type_wrapper(void *out_parameters_ptr)
{
    *(Parameters *)out_parameters_ptr = default_parameters();
}

extern "C" void initialize_state_type_wrapper(void *parameters_ptr,
                                              void *out_initial_state_ptr,
                                              unsigned int num_channels,
                                              float sample_rate, void *allocator)
{
    *(State *)out_initial_state_ptr = initialize_state(
        *(Parameters *)parameters_ptr, num_channels, sample_rate, allocator);
}

// Runtime_No_Error = 0 (ref errors.inc:22).  The oracle's allocator never
// fails, so the longjmp branch of the reference wrapper is unreachable.
extern "C" int initialize_state_error_wrapper(void *parameters_ptr,
                                              void *out_initial_state_ptr,
                                              unsigned int num_channels,
                                              float sample_rate, void *allocator)
{
    initialize_state_type_wrapper(parameters_ptr, out_initial_state_ptr,
                                  num_channels, sample_rate, allocator);
    return 0;
}

extern "C" unsigned long ref_sizeof_parameters(void) { return sizeof(Parameters); }
extern "C" unsigned long ref_sizeof_state(void) { return sizeof(State); }
