# CMake package "SEAL" 3.6 for the MI355X engine.  The reference's callers consume SEAL as
#   find_package(SEAL 3.6 REQUIRED) ... target_link_libraries(<t> SEAL::seal)
# (cnn_ckks/CMakeLists.txt:11,60).  Pointing CMAKE_PREFIX_PATH (or SEAL_DIR) here resolves
# SEAL::seal to libmhe_seal.so (+ libmhe.so) and the seal/seal.h headers of this package.
get_filename_component(_MHE_PREFIX "${CMAKE_CURRENT_LIST_DIR}/../../.." ABSOLUTE)

if(NOT TARGET SEAL::seal)
    if(NOT EXISTS "${_MHE_PREFIX}/libmhe_seal.so")
        set(SEAL_FOUND FALSE)
        set(SEAL_NOT_FOUND_MESSAGE "libmhe_seal.so not built: run make -C ${_MHE_PREFIX}/seal")
        return()
    endif()
    add_library(SEAL::seal SHARED IMPORTED)
    set_target_properties(SEAL::seal PROPERTIES
        IMPORTED_LOCATION "${_MHE_PREFIX}/libmhe_seal.so"
        INTERFACE_INCLUDE_DIRECTORIES "${_MHE_PREFIX}/include"
        INTERFACE_LINK_LIBRARIES "${_MHE_PREFIX}/libmhe.so"
        INTERFACE_COMPILE_FEATURES cxx_std_17)
    # the reference links the static archive name directly in places (gpt2 link.txt)
    add_library(SEAL::seal_shared ALIAS SEAL::seal)
endif()

set(SEAL_FOUND TRUE)
set(SEAL_VERSION 3.6.6)
set(SEAL_USE_MSGSL OFF)
set(SEAL_USE_ZLIB OFF)
set(SEAL_USE_ZSTD OFF)
